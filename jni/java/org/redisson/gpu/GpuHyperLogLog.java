/*
 * RHyperLogLog on the GPU: the object Redisson.getHyperLogLog (Redisson.java:276-283)
 * returns when GPU sketches are enabled.  The executor arrives through the
 * constructor as for every Redisson object (RedissonObject.java:34-48); the
 * public interface is unchanged.  add/addAll/count/countWith/mergeWith and their
 * async twins (RedissonHyperLogLog.java:40-97) run on librsketch, addressed by
 * name in the context's keyspace (two instances of one name are one sketch;
 * count of a name nobody wrote is 0 and creates nothing, as PFCOUNT).
 *
 * addAll implements the INTENDED "PFADD key e1..en": the fork passes the name
 * twice through varargs (RedissonHyperLogLog.java:70-76) and so adds one element.
 *
 * The key lives in GPU memory, not in Redis: delete / isExists / rename /
 * renamenx act on the GPU keyspace; a TTL cannot be honoured, so expire /
 * expireAt fail (UnsupportedOperationException) instead of being silently
 * dropped, clearExpire answers false and remainTimeToLive -1 (no TTL, as
 * PERSIST / PTTL answer for a key without one); move / migrate (other Redis
 * databases or hosts) fail likewise.
 */
package org.redisson.gpu;

import java.util.Collection;
import java.util.Collections;
import java.util.Date;
import java.util.concurrent.TimeUnit;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

import org.redisson.RedissonHyperLogLog;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandAsyncExecutor;

public class GpuHyperLogLog<V> extends RedissonHyperLogLog<V> {

    private final GpuSketchContext gpu;
    private final Codec valueCodec;

    public GpuHyperLogLog(Codec codec, CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        super(codec, commandExecutor, name);
        this.valueCodec = codec;
        this.gpu = gpu;
    }

    public GpuHyperLogLog(CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        this(commandExecutor.getConnectionManager().getCodec(), commandExecutor, name, gpu);
    }

    private String[] withSelf(String... others) {
        String[] names = new String[others.length + 1];
        names[0] = getName();
        System.arraycopy(others, 0, names, 1, others.length);
        return names;
    }

    @Override
    public boolean add(V obj) {
        KeyBuffer kb = KeyBuffer.encodeOne(valueCodec, obj);
        return RSketchNative.hllAdd(gpu.space, getName(), kb.bytes, kb.offsets, 1);
    }

    @Override
    public boolean addAll(Collection<V> objects) {
        KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
        return RSketchNative.hllAdd(gpu.space, getName(), kb.bytes, kb.offsets, kb.n);
    }

    /* n x PFADD in input order (the RBatch form): one reply per element. */
    public boolean[] addEach(Collection<V> objects) {
        KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
        return RSketchNative.hllAddEach(gpu.space, getName(), kb.bytes, kb.offsets, kb.n);
    }

    @Override
    public long count() {
        return RSketchNative.hllCount(gpu.space, getName());
    }

    @Override
    public long countWith(String... otherLogNames) {
        return RSketchNative.hllCountWith(gpu.space, withSelf(otherLogNames));
    }

    @Override
    public void mergeWith(String... otherLogNames) {
        RSketchNative.hllMergeWith(gpu.space, getName(), otherLogNames);
    }

    @Override
    public Future<Boolean> addAsync(V obj) {
        return addAllAsync(Collections.singletonList(obj));
    }

    @Override
    public Future<Boolean> addAllAsync(Collection<V> objects) {
        Promise<Boolean> p = gpu.newPromise();
        try {
            KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
            RSketchNative.hllAddAsync(gpu.space, getName(), kb.bytes, kb.offsets, kb.n, gpu.completion(p));
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Long> countAsync() {
        Promise<Long> p = gpu.newPromise();
        try {
            RSketchNative.hllCountAsync(gpu.space, getName(), gpu.completion(p));
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Long> countWithAsync(String... otherLogNames) {
        Promise<Long> p = gpu.newPromise();
        try {
            RSketchNative.hllCountWithAsync(gpu.space, withSelf(otherLogNames), gpu.completion(p));
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    @Override
    public Future<Void> mergeWithAsync(String... otherLogNames) {
        Promise<Void> p = gpu.newPromise();
        try {
            RSketchNative.hllMergeWithAsync(gpu.space, getName(), otherLogNames, gpu.completion(p));
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    // ---------------------------------------------------------------- keyspace
    @Override
    public Future<Boolean> deleteAsync() {
        Promise<Boolean> p = gpu.newPromise();
        try {
            p.setSuccess(gpu.delete(getName()));
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
