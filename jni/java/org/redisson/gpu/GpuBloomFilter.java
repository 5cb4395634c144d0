/*
 * RBloomFilter on the GPU (Redisson.getBloomFilter, Redisson.java:525-532).
 * Same sizing (optimalNumOfBits / optimalNumOfHashFunctions, MAX_SIZE,
 * RedissonBloomFilter.java:52,69-78,223-229), same hash scheme (xx_r39 +
 * farmUo, (h & Long.MAX_VALUE) % size, :116-131), same replies: add() is true
 * iff one of the first k-1 SETBITs found its bit clear (:100-107), contains()
 * is the AND of the first k-1 GETBITs (:147-168), count() the BITCOUNT
 * formula (:188-199).
 *
 * The filter and its {name}__config live in the context's keyspace
 * (jni/rsketch_shim.h), addressed by name: tryInit stores size, k,
 * expectedInsertions and falseProbability there; every getter reads them
 * back and throws IllegalStateException("Bloom filter is not initialized!")
 * when nobody initialised the name (:258-287); a second getBloomFilter(name)
 * instance sees the first one's size and k.  Like the reference, an instance
 * caches size / hashIterations (:54-55, read when 0); a call made with a
 * stale pair (another client deleted and re-initialised the filter) is
 * refused with RedisException "Bloom filter config has been changed" and
 * retried after re-reading the config (:108-112, :162-166) -- the reference
 * retries with the stale pair; re-reading is what its guard intends.
 */
package org.redisson.gpu;

import java.util.Collection;
import java.util.Date;
import java.util.concurrent.TimeUnit;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

import org.redisson.RedissonBloomFilter;
import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandExecutor;

public class GpuBloomFilter<T> extends RedissonBloomFilter<T> {

    private static final String CONFIG_CHANGED = "Bloom filter config has been changed";

    private final GpuSketchContext gpu;
    private final Codec valueCodec;
    private volatile long size;
    private volatile int hashIterations;

    public GpuBloomFilter(Codec codec, CommandExecutor commandExecutor, String name, GpuSketchContext gpu) {
        super(codec, commandExecutor, name);
        this.valueCodec = codec;
        this.gpu = gpu;
    }

    /* HGETALL {name}__config: {size, hashIterations, expectedInsertions}, falseProbability. */
    private long[] config(double[] fpp) {
        long[] cfg = new long[3];
        RSketchNative.bloomConfig(gpu.space, getName(), cfg, fpp);  // IllegalStateException if absent
        return cfg;
    }

    private void readConfig() {
        long[] cfg = config(null);
        hashIterations = (int) cfg[1];
        size = cfg[0];
    }

    @Override
    public boolean tryInit(long expectedInsertions, double falseProbability) {
        long[] cfg = new long[3];
        boolean created = RSketchNative.bloomTryInit(gpu.space, getName(), expectedInsertions, falseProbability, cfg,
                null);
        hashIterations = (int) cfg[1];  // the config in force: ours, or the existing filter's
        size = cfg[0];
        return created;
    }

    /* One native call for a whole batch (the Redis path: k SETBITs per element),
     * with the reference's config guard and retry. */
    public boolean[] addAll(Collection<T> objects) {
        return batch(KeyBuffer.encode(valueCodec, objects), true);
    }

    public boolean[] containsAll(Collection<T> objects) {
        return batch(KeyBuffer.encode(valueCodec, objects), false);
    }

    private boolean[] batch(KeyBuffer kb, boolean add) {
        while (true) {
            if (size == 0) {
                readConfig();
            }
            long s = size;
            int k = hashIterations;
            try {
                return add ? RSketchNative.bloomAdd(gpu.space, getName(), s, k, kb.bytes, kb.offsets, kb.n)
                           : RSketchNative.bloomContains(gpu.space, getName(), s, k, kb.bytes, kb.offsets, kb.n);
            } catch (RedisException e) {
                if (e.getMessage() == null || !e.getMessage().contains(CONFIG_CHANGED)) {
                    throw e;
                }
                size = 0;  // re-read {name}__config
            }
        }
    }

    @Override
    public boolean add(T object) {
        return batch(KeyBuffer.encodeOne(valueCodec, object), true)[0];
    }

    @Override
    public boolean contains(T object) {
        return batch(KeyBuffer.encodeOne(valueCodec, object), false)[0];
    }

    /* Futures of a batch add / contains, completed by the library's callback. */
    public Future<boolean[]> addAllAsync(Collection<T> objects) {
        return batchAsync(objects, true);
    }

    public Future<boolean[]> containsAllAsync(Collection<T> objects) {
        return batchAsync(objects, false);
    }

    private Future<boolean[]> batchAsync(Collection<T> objects, boolean add) {
        Promise<boolean[]> p = gpu.newPromise();
        try {
            KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
            if (size == 0) {
                readConfig();
            }
            if (add) {
                RSketchNative.bloomAddAsync(gpu.space, getName(), size, hashIterations, kb.bytes, kb.offsets, kb.n,
                        gpu.completion(p));
            } else {
                RSketchNative.bloomContainsAsync(gpu.space, getName(), size, hashIterations, kb.bytes, kb.offsets, kb.n,
                        gpu.completion(p));
            }
        } catch (RedisException e) {
            if (e.getMessage() != null && e.getMessage().contains(CONFIG_CHANGED)) {
                size = 0;  // the config moved on: issue again with the new one
                return batchAsync(objects, add);
            }
            p.tryFailure(e);
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public int count() {
        readConfig();  // as the reference reads the config with BITCOUNT (:188-199)
        return RSketchNative.bloomCount(gpu.space, getName());
    }

    @Override
    public long getSize() {
        return config(null)[0];
    }

    @Override
    public int getHashIterations() {
        return (int) config(null)[1];
    }

    @Override
    public long getExpectedInsertions() {
        return config(null)[2];
    }

    @Override
    public double getFalseProbability() {
        double[] fpp = new double[1];
        config(fpp);
        return fpp[0];
    }

    // ---------------------------------------------------------------- keyspace
    @Override
    public Future<Boolean> deleteAsync() {
        Promise<Boolean> p = gpu.newPromise();
        try {
            p.setSuccess(gpu.delete(getName()));  // the filter and its {name}__config
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Boolean> isExistsAsync() {
        Promise<Boolean> p = gpu.newPromise();
        p.setSuccess(gpu.type(getName()) != RSketchNative.NONE);
        return p;
    }

    @Override
    public Future<Void> renameAsync(String newName) {
        Promise<Void> p = gpu.newPromise();
        try {
            GpuKeyspace.rename(gpu, getName(), newName, false);
            p.setSuccess(null);
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Boolean> renamenxAsync(String newName) {
        Promise<Boolean> p = gpu.newPromise();
        try {
            p.setSuccess(GpuKeyspace.rename(gpu, getName(), newName, true));
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Boolean> expireAsync(long timeToLive, TimeUnit timeUnit) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> expireAtAsync(long timestamp) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> expireAtAsync(Date timestamp) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> clearExpireAsync() {
        Promise<Boolean> p = gpu.newPromise();
        p.setSuccess(Boolean.FALSE);
        return p;
    }

    @Override
    public Future<Long> remainTimeToLiveAsync() {
        Promise<Long> p = gpu.newPromise();
        p.setSuccess(Long.valueOf(-1));
        return p;
    }

    @Override
    public Future<Boolean> moveAsync(int database) {
        return gpu.failed(GpuKeyspace.notOnGpu("move"));
    }

    @Override
    public Future<Void> migrateAsync(String host, int port, int database) {
        return gpu.failed(GpuKeyspace.notOnGpu("migrate"));
    }
}
