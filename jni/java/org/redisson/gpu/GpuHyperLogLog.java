/*
 * RHyperLogLog on the GPU: the object Redisson.getHyperLogLog (Redisson.java:276-283)
 * returns when GPU sketches are enabled.  The executor arrives through the
 * constructor as for every Redisson object (RedissonObject.java:34-48); the
 * public interface is unchanged.  add/addAll/count/countWith/mergeWith and their
 * async twins (RedissonHyperLogLog.java:40-97) run on librsketch; expire/rename
 * and the other RExpirable calls stay with the Redis executor.
 *
 * addAll implements the INTENDED "PFADD key e1..en": the fork passes the name
 * twice through varargs (RedissonHyperLogLog.java:70-76) and so adds one element.
 */
package org.redisson.gpu;

import java.util.Arrays;
import java.util.Collection;
import java.util.concurrent.Callable;

import io.netty.util.concurrent.Future;

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

    private Callable<Boolean> addTask(final Collection<V> objects) {
        return new Callable<Boolean>() {
            public Boolean call() {
                KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
                return RSketchNative.hllAdd(gpu.hll(getName()), 0, kb.bytes, kb.offsets, kb.n);
            }
        };
    }

    private Callable<Long> countTask(final String... others) {
        return new Callable<Long>() {
            public Long call() {
                if (others.length == 0) {
                    return RSketchNative.hllCount(gpu.hll(getName()), 0);
                }
                long[] hs = new long[others.length + 1];
                long[] ids = new long[others.length + 1];
                hs[0] = gpu.hll(getName());
                for (int i = 0; i < others.length; i++) {
                    hs[i + 1] = gpu.hll(others[i]);
                }
                return RSketchNative.hllCountUnion(hs, ids);
            }
        };
    }

    private Callable<Void> mergeTask(final String... others) {
        return new Callable<Void>() {
            public Void call() {
                long[] hs = new long[others.length];
                long[] ids = new long[others.length];
                for (int i = 0; i < others.length; i++) {
                    hs[i] = gpu.hll(others[i]);
                }
                RSketchNative.hllMerge(gpu.hll(getName()), 0, hs, ids);
                return null;
            }
        };
    }

    @Override
    public boolean add(V obj) {
        return gpu.call(addTask(Arrays.asList(obj)));
    }

    @Override
    public boolean addAll(Collection<V> objects) {
        return gpu.call(addTask(objects));
    }

    @Override
    public long count() {
        return gpu.call(countTask());
    }

    @Override
    public long countWith(String... otherLogNames) {
        return gpu.call(countTask(otherLogNames));
    }

    @Override
    public void mergeWith(String... otherLogNames) {
        gpu.call(mergeTask(otherLogNames));
    }

    @Override
    public Future<Boolean> addAsync(V obj) {
        return gpu.callAsync(addTask(Arrays.asList(obj)));
    }

    @Override
    public Future<Boolean> addAllAsync(Collection<V> objects) {
        return gpu.callAsync(addTask(objects));
    }

    @Override
    public Future<Long> countAsync() {
        return gpu.callAsync(countTask());
    }

    @Override
    public Future<Long> countWithAsync(String... otherLogNames) {
        return gpu.callAsync(countTask(otherLogNames));
    }

    @Override
    public Future<Void> mergeWithAsync(String... otherLogNames) {
        return gpu.callAsync(mergeTask(otherLogNames));
    }

    @Override
    public boolean delete() {
        return gpu.call(new Callable<Boolean>() {
            public Boolean call() {
                RSketchNative.hllDelete(gpu.hll(getName()), 0);
                return true;
            }
        });
    }
}
