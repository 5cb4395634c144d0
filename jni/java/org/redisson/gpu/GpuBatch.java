/*
 * RBatch for GPU sketches (RedissonBatch.java:55-83 getHyperLogLog, :226-233
 * execute; RedissonBatch on Redis pipelines the queued commands in one flush).
 * getHyperLogLog(name) / getBitSet(name) (:191) return async objects whose calls are queued and
 * answered by execute(), in the order they were queued: every run of queued
 * add()s -- whatever names they go to -- becomes ONE native call
 * (rsk_shim_batch_hll_add: one rsk_hll_add_each per name, replies in input
 * order), every run of queued SETBITs on one name with one value becomes ONE
 * rsk_bitset_setbits call; the other calls run in their queue position.  executeAsync() does the
 * same off the calling thread's future.  The futures the queued calls return
 * complete with their replies when execute() runs.
 */
package org.redisson.gpu;

import java.util.ArrayList;
import java.util.BitSet;
import java.util.Collection;
import java.util.List;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

import org.redisson.client.codec.Codec;
import org.redisson.core.RBitSetAsync;
import org.redisson.core.RHyperLogLogAsync;

public final class GpuBatch {

    private final GpuSketchContext gpu;
    private final List<Op> ops = new ArrayList<Op>();
    private boolean executed;

    GpuBatch(GpuSketchContext gpu) {
        this.gpu = gpu;
    }

    private abstract static class Op {
        final Promise<Object> promise;

        Op(Promise<Object> promise) {
            this.promise = promise;
        }
    }

    private static final class AddOp extends Op {
        final String name;
        final byte[] element;

        AddOp(Promise<Object> p, String name, byte[] element) {
            super(p);
            this.name = name;
            this.element = element;
        }
    }

    /* setAsync(bit[, value]) / clearAsync(bit): a run of them on one name with
     * one value becomes one SETBIT-many call (rsk_bitset_setbits). */
    private static final class SetBitOp extends Op {
        final String name;
        final long index;
        final boolean value;

        SetBitOp(Promise<Object> p, String name, long index, boolean value) {
            super(p);
            this.name = name;
            this.index = index;
            this.value = value;
        }
    }

    private static final class CallOp extends Op {
        final java.util.concurrent.Callable<Object> call;

        CallOp(Promise<Object> p, java.util.concurrent.Callable<Object> call) {
            super(p);
            this.call = call;
        }
    }

    private synchronized <R> Future<R> queue(Op op) {
        if (executed) {
            throw new IllegalStateException("Batch already executed!");
        }
        ops.add(op);
        @SuppressWarnings("unchecked")
        Future<R> f = (Future<R>) (Future<?>) op.promise;
        return f;
    }

    public <V> RHyperLogLogAsync<V> getHyperLogLog(String name, Codec codec) {
        return new BatchHyperLogLog<V>(name, codec);
    }

    /* RBatch.getBitSet (RedissonBatch.java:191): on a Bloom filter's name it
     * reads and writes the filter's bits, as GpuBitSet does. */
    public RBitSetAsync getBitSet(String name) {
        return new BatchBitSet(name);
    }

    /* Runs the queued calls; their replies, in queue order (RBatch.execute). */
    public synchronized List<?> execute() {
        if (executed) {
            throw new IllegalStateException("Batch already executed!");
        }
        executed = true;
        List<Object> results = new ArrayList<Object>(ops.size());
        int i = 0;
        while (i < ops.size()) {
            if (ops.get(i) instanceof AddOp) {
                int j = i;
                while (j < ops.size() && ops.get(j) instanceof AddOp) {
                    j++;
                }
                runAdds(ops.subList(i, j));
                i = j;
            } else if (ops.get(i) instanceof SetBitOp) {
                SetBitOp first = (SetBitOp) ops.get(i);
                int j = i;
                while (j < ops.size() && ops.get(j) instanceof SetBitOp && ((SetBitOp) ops.get(j)).name.equals(first.name)
                        && ((SetBitOp) ops.get(j)).value == first.value) {
                    j++;
                }
                runSetBits(ops.subList(i, j));
                i = j;
            } else {
                CallOp c = (CallOp) ops.get(i++);
                try {
                    c.promise.setSuccess(c.call.call());
                } catch (Exception e) {
                    c.promise.setFailure(e);
                }
            }
        }
        for (Op op : ops) {
            if (!op.promise.isSuccess()) {
                Throwable t = op.promise.cause();
                throw t instanceof RuntimeException ? (RuntimeException) t : new IllegalStateException(t);
            }
            results.add(op.promise.getNow());
        }
        return results;
    }

    public Future<List<?>> executeAsync() {
        Promise<List<?>> p = gpu.newPromise();
        try {
            p.setSuccess(execute());
        } catch (RuntimeException e) {
            p.setFailure(e);
        }
        return p;
    }

    /* One native call for a run of queued add()s across names. */
    private void runAdds(List<Op> run) {
        List<String> names = new ArrayList<String>();
        int[] nameOf = new int[run.size()];
        List<byte[]> elements = new ArrayList<byte[]>(run.size());
        for (int q = 0; q < run.size(); q++) {
            AddOp a = (AddOp) run.get(q);
            int at = names.indexOf(a.name);
            if (at < 0) {
                at = names.size();
                names.add(a.name);
            }
            nameOf[q] = at;
            elements.add(a.element);
        }
        try {
            KeyBuffer kb = KeyBuffer.ofEncoded(elements);
            boolean[] replies = RSketchNative.batchHllAdd(gpu.space, names.toArray(new String[names.size()]), nameOf,
                    kb.bytes, kb.offsets, kb.n);
            for (int q = 0; q < run.size(); q++) {
                run.get(q).promise.setSuccess(Boolean.valueOf(replies[q]));
            }
        } catch (RuntimeException e) {
            for (Op op : run) {
                op.promise.setFailure(e);
            }
        }
    }

    /* Largest SETBIT offset Redis accepts (512 MB strings: 2^32 - 1 bits), as
     * the shim's check (rsketch_shim.c offsets_ok). */
    private static final long MAX_BIT_OFFSET = 4294967295L;

    /* A pipeline fails only the SETBITs Redis rejects (offset out of range, each
     * with Redis's error) and applies the others: they go in one native call. */
    private void runSetBits(List<Op> run) {
        SetBitOp first = (SetBitOp) run.get(0);
        List<Op> good = new ArrayList<Op>(run.size());
        for (Op op : run) {
            long index = ((SetBitOp) op).index;
            if (index < 0 || index > MAX_BIT_OFFSET) {
                op.promise.setFailure(new org.redisson.client.RedisException(
                        "ERR bit offset is not an integer or out of range"));
            } else {
                good.add(op);
            }
        }
        if (good.isEmpty()) {
            return;
        }
        long[] indexes = new long[good.size()];
        for (int q = 0; q < good.size(); q++) {
            indexes[q] = ((SetBitOp) good.get(q)).index;
        }
        try {
            RSketchNative.bitsetSetBits(gpu.space, first.name, indexes, first.value);
            for (Op op : good) {
                op.promise.setSuccess(null);
            }
        } catch (RuntimeException e) {
            for (Op op : good) {
                op.promise.setFailure(e);
            }
        }
    }

    private final class BatchBitSet implements RBitSetAsync {
        private final String name;

        BatchBitSet(String name) {
            this.name = name;
        }

        private Promise<Object> promise() {
            return gpu.newPromise();
        }

        private <R> Future<R> call(java.util.concurrent.Callable<Object> c) {
            return queue(new CallOp(promise(), c));
        }

        private <R> Future<R> op(final int op, final String... others) {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    RSketchNative.bitsetOp(gpu.space, name, op, others);
                    return null;
                }
            });
        }

        public String getName() {
            return name;
        }

        public Future<byte[]> toByteArrayAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return RSketchNative.bitsetGet(gpu.space, name);
                }
            });
        }

        public Future<Long> lengthAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Long.valueOf(RSketchNative.bitsetLength(gpu.space, name));
                }
            });
        }

        public Future<Void> setAsync(final long fromIndex, final long toIndex, final boolean value) {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    RSketchNative.bitsetSetRange(gpu.space, name, fromIndex, toIndex, value);
                    return null;
                }
            });
        }

        public Future<Void> clearAsync(long fromIndex, long toIndex) {
            return setAsync(fromIndex, toIndex, false);
        }

        public Future<Void> setAsync(long fromIndex, long toIndex) {
            return setAsync(fromIndex, toIndex, true);
        }

        public Future<Void> setAsync(BitSet bs) {
            final byte[] bytes = GpuBitSet.encode(bs);
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    RSketchNative.bitsetSet(gpu.space, name, bytes);
                    return null;
                }
            });
        }

        public Future<Void> notAsync() {
            return op(RSketchNative.BITOP_NOT);
        }

        public Future<Integer> sizeAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Integer.valueOf((int) (RSketchNative.bitsetStrlen(gpu.space, name) * 8));
                }
            });
        }

        public Future<Boolean> getAsync(final long bitIndex) {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Boolean.valueOf(RSketchNative.bitsetGetBits(gpu.space, name, new long[] {bitIndex})[0]);
                }
            });
        }

        public Future<Void> setAsync(long bitIndex) {
            return setAsync(bitIndex, true);
        }

        public Future<Void> setAsync(long bitIndex, boolean value) {
            return queue(new SetBitOp(promise(), name, bitIndex, value));
        }

        public Future<Long> cardinalityAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Long.valueOf(RSketchNative.bitsetCardinality(gpu.space, name));
                }
            });
        }

        public Future<Void> clearAsync(long bitIndex) {
            return setAsync(bitIndex, false);
        }

        public Future<Void> clearAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    RSketchNative.bitsetClear(gpu.space, name);
                    return null;
                }
            });
        }

        public Future<Void> orAsync(String... bitSetNames) {
            return op(RSketchNative.BITOP_OR, bitSetNames);
        }

        public Future<Void> andAsync(String... bitSetNames) {
            return op(RSketchNative.BITOP_AND, bitSetNames);
        }

        public Future<Void> xorAsync(String... bitSetNames) {
            return op(RSketchNative.BITOP_XOR, bitSetNames);
        }

        public Future<Boolean> deleteAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Boolean.valueOf(RSketchNative.bitsetClear(gpu.space, name));
                }
            });
        }

        public Future<Boolean> isExistsAsync() {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return Boolean.valueOf(RSketchNative.bitsetStrlen(gpu.space, name) > 0);
                }
            });
        }

        public Future<Void> renameAsync(final String newName) {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    GpuKeyspace.rename(gpu, name, newName, false);
                    return null;
                }
            });
        }

        public Future<Boolean> renamenxAsync(final String newName) {
            return call(new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return GpuKeyspace.rename(gpu, name, newName, true);
                }
            });
        }

        public Future<Void> migrateAsync(String host, int port, int database) {
            return gpu.failed(GpuKeyspace.notOnGpu("migrate"));
        }

        public Future<Boolean> moveAsync(int database) {
            return gpu.failed(GpuKeyspace.notOnGpu("move"));
        }

        public Future<Boolean> expireAsync(long timeToLive, java.util.concurrent.TimeUnit timeUnit) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> expireAtAsync(long timestamp) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> expireAtAsync(java.util.Date timestamp) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> clearExpireAsync() {
            Promise<Boolean> p = gpu.newPromise();
            p.setSuccess(Boolean.FALSE);
            return p;
        }

        public Future<Long> remainTimeToLiveAsync() {
            Promise<Long> p = gpu.newPromise();
            p.setSuccess(Long.valueOf(-1));
            return p;
        }
    }

    private final class BatchHyperLogLog<V> implements RHyperLogLogAsync<V> {
        private final String name;
        private final Codec codec;

        BatchHyperLogLog(String name, Codec codec) {
            this.name = name;
            this.codec = codec;
        }

        private Promise<Object> promise() {
            return gpu.newPromise();
        }

        public Future<Boolean> addAsync(V obj) {
            return queue(new AddOp(promise(), name, KeyBuffer.encodeElement(codec, obj)));
        }

        public Future<Boolean> addAllAsync(final Collection<V> objects) {
            final Codec c = codec;
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    KeyBuffer kb = KeyBuffer.encode(c, objects);
                    return RSketchNative.hllAdd(gpu.space, name, kb.bytes, kb.offsets, kb.n);
                }
            }));
        }

        public Future<Long> countAsync() {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return RSketchNative.hllCount(gpu.space, name);
                }
            }));
        }

        public Future<Long> countWithAsync(final String... otherLogNames) {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    String[] names = new String[otherLogNames.length + 1];
                    names[0] = name;
                    System.arraycopy(otherLogNames, 0, names, 1, otherLogNames.length);
                    return RSketchNative.hllCountWith(gpu.space, names);
                }
            }));
        }

        public Future<Void> mergeWithAsync(final String... otherLogNames) {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    RSketchNative.hllMergeWith(gpu.space, name, otherLogNames);
                    return null;
                }
            }));
        }

        public String getName() {
            return name;
        }

        public Future<Boolean> deleteAsync() {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return gpu.delete(name);
                }
            }));
        }

        public Future<Boolean> isExistsAsync() {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return gpu.type(name) != RSketchNative.NONE;
                }
            }));
        }

        public Future<Void> renameAsync(final String newName) {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    GpuKeyspace.rename(gpu, name, newName, false);
                    return null;
                }
            }));
        }

        public Future<Boolean> renamenxAsync(final String newName) {
            return queue(new CallOp(promise(), new java.util.concurrent.Callable<Object>() {
                public Object call() {
                    return GpuKeyspace.rename(gpu, name, newName, true);
                }
            }));
        }

        public Future<Void> migrateAsync(String host, int port, int database) {
            return gpu.failed(GpuKeyspace.notOnGpu("migrate"));
        }

        public Future<Boolean> moveAsync(int database) {
            return gpu.failed(GpuKeyspace.notOnGpu("move"));
        }

        public Future<Boolean> expireAsync(long timeToLive, java.util.concurrent.TimeUnit timeUnit) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> expireAtAsync(long timestamp) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> expireAtAsync(java.util.Date timestamp) {
            return gpu.failed(GpuKeyspace.noTtl());
        }

        public Future<Boolean> clearExpireAsync() {
            Promise<Boolean> p = gpu.newPromise();
            p.setSuccess(Boolean.FALSE);
            return p;
        }

        public Future<Long> remainTimeToLiveAsync() {
            Promise<Long> p = gpu.newPromise();
            p.setSuccess(Long.valueOf(-1));
            return p;
        }
    }
}
