/*
 * RBitSetReactive on the GPU keyspace: what RedissonReactive.getBitSet
 * (src/main/java/org/redisson/RedissonReactive.java:264-266) returns when GPU
 * sketches are enabled.  The reference's RedissonBitSetReactive
 * (reactive/RedissonBitSetReactive.java:29-113) wraps a RedissonBitSet and
 * returns reactive(instance.xxxAsync()); this wraps a GpuBitSet of the same
 * name -- so a name holding a GPU Bloom filter reads the filter's bits, as
 * getBitSet(name) does on the blocking client -- and wraps its futures as the
 * reactive executor wraps a reply's (GpuReactive).  asBitSet is GET decoded
 * by BitSetCodec.fromByteArrayReverse (client/codec/BitSetCodec.java:39-47:
 * bit i set iff byte i/8 has 0x80 >> i%8); a missing string emits nothing, as
 * a null GET reply does.
 */
package org.redisson.gpu;

import java.util.BitSet;
import java.util.Date;
import java.util.concurrent.TimeUnit;

import org.reactivestreams.Publisher;
import org.redisson.api.RBitSetReactive;
import org.redisson.command.CommandAsyncExecutor;

public class GpuBitSetReactive implements RBitSetReactive {

    private final GpuBitSet instance;
    private final GpuSketchContext gpu;

    public GpuBitSetReactive(CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        this.instance = new GpuBitSet(commandExecutor, name, gpu);
        this.gpu = gpu;
    }

    static BitSet fromByteArrayReverse(byte[] bytes) {
        BitSet bits = new BitSet();
        for (int i = 0; i < bytes.length * 8; i++) {
            if ((bytes[i >>> 3] & (0x80 >>> (i & 7))) != 0) {
                bits.set(i);
            }
        }
        return bits;
    }

    @Override
    public String getName() {
        return instance.getName();
    }

    @Override
    public Publisher<BitSet> asBitSet() {
        return GpuReactive.publisher(GpuReactive.map(gpu, instance.toByteArrayAsync(), new GpuReactive.Map<byte[], BitSet>() {
            BitSet apply(byte[] b) {
                return fromByteArrayReverse(b);
            }
        }));
    }

    @Override
    public Publisher<byte[]> toByteArray() {
        return GpuReactive.publisher(instance.toByteArrayAsync());
    }

    @Override
    public Publisher<Long> length() {
        return GpuReactive.publisher(instance.lengthAsync());
    }

    @Override
    public Publisher<Void> set(long fromIndex, long toIndex, boolean value) {
        return GpuReactive.publisher(instance.setAsync(fromIndex, toIndex, value));
    }

    @Override
    public Publisher<Void> clear(long fromIndex, long toIndex) {
        return GpuReactive.publisher(instance.clearAsync(fromIndex, toIndex));
    }

    @Override
    public Publisher<Void> set(BitSet bs) {
        return GpuReactive.publisher(instance.setAsync(bs));
    }

    @Override
    public Publisher<Void> not() {
        return GpuReactive.publisher(instance.notAsync());
    }

    @Override
    public Publisher<Void> set(long fromIndex, long toIndex) {
        return GpuReactive.publisher(instance.setAsync(fromIndex, toIndex));
    }

    @Override
    public Publisher<Integer> size() {
        return GpuReactive.publisher(instance.sizeAsync());
    }

    @Override
    public Publisher<Boolean> get(long bitIndex) {
        return GpuReactive.publisher(instance.getAsync(bitIndex));
    }

    @Override
    public Publisher<Void> set(long bitIndex) {
        return GpuReactive.publisher(instance.setAsync(bitIndex));
    }

    @Override
    public Publisher<Void> set(long bitIndex, boolean value) {
        return GpuReactive.publisher(instance.setAsync(bitIndex, value));
    }

    @Override
    public Publisher<Long> cardinality() {
        return GpuReactive.publisher(instance.cardinalityAsync());
    }

    @Override
    public Publisher<Void> clear(long bitIndex) {
        return GpuReactive.publisher(instance.clearAsync(bitIndex));
    }

    @Override
    public Publisher<Void> clear() {
        return GpuReactive.publisher(instance.clearAsync());
    }

    @Override
    public Publisher<Void> or(String... bitSetNames) {
        return GpuReactive.publisher(instance.orAsync(bitSetNames));
    }

    @Override
    public Publisher<Void> and(String... bitSetNames) {
        return GpuReactive.publisher(instance.andAsync(bitSetNames));
    }

    @Override
    public Publisher<Void> xor(String... bitSetNames) {
        return GpuReactive.publisher(instance.xorAsync(bitSetNames));
    }

    // ---------------------------------------------------------------- keyspace
    @Override
    public Publisher<Boolean> delete() {
        return GpuReactive.publisher(instance.deleteAsync());
    }

    @Override
    public Publisher<Boolean> isExists() {
        return GpuReactive.publisher(instance.isExistsAsync());
    }

    @Override
    public Publisher<Void> rename(String newName) {
        return GpuReactive.publisher(instance.renameAsync(newName));
    }

    @Override
    public Publisher<Boolean> renamenx(String newName) {
        return GpuReactive.publisher(instance.renamenxAsync(newName));
    }

    @Override
    public Publisher<Boolean> expire(long timeToLive, TimeUnit timeUnit) {
        return GpuReactive.publisher(instance.expireAsync(timeToLive, timeUnit));
    }

    @Override
    public Publisher<Boolean> expireAt(Date timestamp) {
        return GpuReactive.publisher(instance.expireAtAsync(timestamp));
    }

    @Override
    public Publisher<Boolean> expireAt(long timestamp) {
        return GpuReactive.publisher(instance.expireAtAsync(timestamp));
    }

    @Override
    public Publisher<Boolean> clearExpire() {
        return GpuReactive.publisher(instance.clearExpireAsync());
    }

    @Override
    public Publisher<Long> remainTimeToLive() {
        return GpuReactive.publisher(instance.remainTimeToLiveAsync());
    }

    @Override
    public Publisher<Boolean> move(int database) {
        return GpuReactive.publisher(instance.moveAsync(database));
    }

    @Override
    public Publisher<Void> migrate(String host, int port, int database) {
        return GpuReactive.publisher(instance.migrateAsync(host, port, database));
    }

    @Override
    public String toString() {
        return instance.toString();
    }
}
