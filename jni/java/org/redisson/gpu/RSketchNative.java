/*
 * Native methods of the GPU sketch engine (librsketch.so) as the JNI glue
 * jni/rsketch_jni.c exports them, over the shim's keyspace (jni/rsketch_shim.h):
 * objects are addressed by NAME in a space (one GPU context + its name ->
 * object registry), exactly as the Redis-backed objects address keys.
 * Key batches are direct buffers (GetDirectBufferAddress, no copy): the
 * codec-encoded elements back to back, and n+1 byte offsets in native order
 * (see KeyBuffer).  Errors arrive as the exceptions the Redis path raises
 * (IllegalArgumentException, IllegalStateException, RedisException).
 */
package org.redisson.gpu;

import java.nio.ByteBuffer;
import java.nio.LongBuffer;
import java.util.concurrent.Executor;

import io.netty.util.concurrent.Promise;

final class RSketchNative {

    static {
        System.loadLibrary("rsketch_jni"); // links librsketch.so
    }

    /* RSK_SHIM_NONE / _HLL / _BLOOM / _BITSET */
    static final int NONE = 0;
    static final int HLL = 1;
    static final int BLOOM = 2;
    static final int BITSET = 3;

    /* completion kinds (rsketch_jni.c) */
    static final int K_BOOL = 0;
    static final int K_LONG = 1;
    static final int K_VOID = 2;
    static final int K_ARRAY = 3;

    private RSketchNative() {
    }

    static native long init(int device, boolean extendedBloom);          // rsk_shim_init
    static native void shutdown(long space);
    static native int type(long space, String name);                      // rsk_shim_lookup
    static native boolean delete(long space, String name);                // DEL name ({name}__config too)
    static native boolean rename(long space, String oldName, String newName, boolean nx); // RENAME / RENAMENX

    static native boolean hllAdd(long space, String name, ByteBuffer keys, LongBuffer offsets, long n);       // PFADD
    static native boolean[] hllAddEach(long space, String name, ByteBuffer keys, LongBuffer offsets, long n); // n x PFADD
    static native long hllCount(long space, String name);                 // PFCOUNT (0 if missing)
    static native long hllCountWith(long space, String[] names);          // PFCOUNT k1..kk
    static native void hllMergeWith(long space, String dst, String[] srcs); // PFMERGE dst src..
    static native boolean[] batchHllAdd(long space, String[] names, int[] nameOf, ByteBuffer keys, LongBuffer offsets,
                                        long n);                          // RBatch of add()s

    static native void hllAddAsync(long space, String name, ByteBuffer keys, LongBuffer offsets, long n,
                                   Completion<Boolean> done);
    static native void hllCountAsync(long space, String name, Completion<Long> done);
    static native void hllCountWithAsync(long space, String[] names, Completion<Long> done);
    static native void hllMergeWithAsync(long space, String dst, String[] srcs, Completion<Void> done);

    /* cfg = {size, hashIterations, expectedInsertions}, fpp = {falseProbability}: the {name}__config hash */
    static native boolean bloomTryInit(long space, String name, long expectedInsertions, double falseProbability,
                                       long[] cfg, double[] fpp);
    static native void bloomConfig(long space, String name, long[] cfg, double[] fpp); // IllegalStateException if absent
    static native boolean[] bloomAdd(long space, String name, long size, int k, ByteBuffer keys, LongBuffer offsets,
                                     long n);
    static native boolean[] bloomContains(long space, String name, long size, int k, ByteBuffer keys,
                                          LongBuffer offsets, long n);
    static native int bloomCount(long space, String name);
    static native void bloomAddAsync(long space, String name, long size, int k, ByteBuffer keys, LongBuffer offsets,
                                     long n, Completion<boolean[]> done);
    static native void bloomContainsAsync(long space, String name, long size, int k, ByteBuffer keys,
                                          LongBuffer offsets, long n, Completion<boolean[]> done);

    /* RBitSet on the keyspace (rsk_shim_bitset_*): a plain string, or the bits of
     * a Bloom filter of that name (Redis keeps them as the string key `name`). */
    static native long bitsetStrlen(long space, String name);                     // STRLEN
    static native byte[] bitsetGet(long space, String name);                      // GET (null: nil)
    static native boolean[] bitsetGetBits(long space, String name, long[] indexes); // GETBIT x n
    static native void bitsetSetBits(long space, String name, long[] indexes, boolean value); // SETBIT x n
    static native void bitsetSetRange(long space, String name, long from, long to, boolean value);
    static native long bitsetCardinality(long space, String name);                // BITCOUNT
    static native long bitsetLength(long space, String name);                     // length()
    static native void bitsetSet(long space, String name, byte[] bytes);          // SET
    static native boolean bitsetClear(long space, String name);                   // DEL (a filter keeps its config)
    static native void bitsetOp(long space, String name, int op, String[] others); // BITOP op name name others

    static final int BITOP_AND = 0;
    static final int BITOP_OR = 1;
    static final int BITOP_XOR = 2;
    static final int BITOP_NOT = 3;

    /* Waits until every call issued on the space so far has completed and its
     * completion has been handed to its executor (rsk_shim_sync). */
    static native void sync(long space);

    /* Delivers completions the library's thread could not (it failed to attach
     * to the JVM); every other native method does this first as well. */
    static native void reap();

    /* One asynchronous call's promise and the executor its listeners run on. */
    static final class Completion<T> {
        final Promise<T> promise;
        final Executor executor;

        Completion(Promise<T> promise, Executor executor) {
            this.promise = promise;
            this.executor = executor;
        }
    }

    /* Called by the JNI glue on the library's completion thread (attached to the
     * JVM as a daemon), in submission order.  It only hands the result to the
     * completion's executor -- the Netty event loop GpuSketchContext pinned, as
     * a Redis reply completes its promise on a connection's event loop
     * (CommandAsyncService.java:86-105) -- so user listeners never run on the
     * library's thread.  An executor that refuses (shut down) completes the
     * promise here instead: a future is never left pending. */
    @SuppressWarnings("unchecked")
    static void complete(Object target, final int kind, final int status, final long value, final boolean[] replies) {
        final Completion<Object> c = (Completion<Object>) target;
        Runnable r = new Runnable() {
            public void run() {
                fulfil(c.promise, kind, status, value, replies);
            }
        };
        try {
            c.executor.execute(r);
        } catch (Throwable t) {  // RejectedExecutionException: the event loop is shutting down
            r.run();
        }
    }

    static void fulfil(Promise<Object> p, int kind, int status, long value, boolean[] replies) {
        try {
            if (status != 0) {
                p.tryFailure(new org.redisson.client.RedisException("GPU call failed with status " + status
                        + (status == 5 ? " (device error: the context is unusable)" : "")));
                return;
            }
            switch (kind) {
                case K_BOOL:
                    p.trySuccess(Boolean.valueOf(value != 0));
                    break;
                case K_LONG:
                    p.trySuccess(Long.valueOf(value));
                    break;
                case K_ARRAY:
                    p.trySuccess(replies);
                    break;
                default:
                    p.trySuccess(null);
                    break;
            }
        } catch (Throwable t) {
            p.tryFailure(t);
        }
    }
}
