/*
 * RHyperLogLogReactive on the GPU keyspace: what RedissonReactive.getHyperLogLog
 * (src/main/java/org/redisson/RedissonReactive.java:146-151) returns when GPU
 * sketches are enabled.  The reference's RedissonHyperLogLogReactive
 * (reactive/RedissonHyperLogLogReactive.java:38-75) sends PFADD / PFCOUNT /
 * PFMERGE through the reactive executor; here every method is the matching
 * asynchronous call of a GpuHyperLogLog of the same name and codec (the same
 * sketch as getHyperLogLog(name) on the blocking client), its future wrapped
 * as the reactive executor wraps a reply's (GpuReactive).  Keyspace methods
 * (delete, rename, TTL, move, migrate) answer as GpuHyperLogLog's do.
 */
package org.redisson.gpu;

import java.util.Collection;
import java.util.Date;
import java.util.concurrent.TimeUnit;

import org.reactivestreams.Publisher;
import org.redisson.api.RHyperLogLogReactive;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandAsyncExecutor;

public class GpuHyperLogLogReactive<V> implements RHyperLogLogReactive<V> {

    private final GpuHyperLogLog<V> instance;

    public GpuHyperLogLogReactive(Codec codec, CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        this.instance = new GpuHyperLogLog<V>(codec, commandExecutor, name, gpu);
    }

    public GpuHyperLogLogReactive(CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        this.instance = new GpuHyperLogLog<V>(commandExecutor, name, gpu);
    }

    @Override
    public String getName() {
        return instance.getName();
    }

    @Override
    public Publisher<Boolean> add(V obj) {
        return GpuReactive.publisher(instance.addAsync(obj));
    }

    @Override
    public Publisher<Boolean> addAll(Collection<V> objects) {
        return GpuReactive.publisher(instance.addAllAsync(objects));
    }

    @Override
    public Publisher<Long> count() {
        return GpuReactive.publisher(instance.countAsync());
    }

    @Override
    public Publisher<Long> countWith(String... otherLogNames) {
        return GpuReactive.publisher(instance.countWithAsync(otherLogNames));
    }

    @Override
    public Publisher<Void> mergeWith(String... otherLogNames) {
        return GpuReactive.publisher(instance.mergeWithAsync(otherLogNames));
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
}
