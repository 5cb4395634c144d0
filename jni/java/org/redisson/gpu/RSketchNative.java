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

import io.netty.util.concurrent.Promise;

final class RSketchNative {

    static {
        System.loadLibrary("rsketch_jni"); // links librsketch.so
    }

    /* RSK_SHIM_NONE / _HLL / _BLOOM */
    static final int NONE = 0;
    static final int HLL = 1;
    static final int BLOOM = 2;

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
                                   Promise<Boolean> promise);
    static native void hllCountAsync(long space, String name, Promise<Long> promise);
    static native void hllCountWithAsync(long space, String[] names, Promise<Long> promise);
    static native void hllMergeWithAsync(long space, String dst, String[] srcs, Promise<Void> promise);

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
                                     long n, Promise<boolean[]> promise);
    static native void bloomContainsAsync(long space, String name, long size, int k, ByteBuffer keys,
                                          LongBuffer offsets, long n, Promise<boolean[]> promise);

    /* Called by the JNI glue from the completion callback (a HIP runtime
     * thread, attached as a daemon): completes the promise; its listeners run
     * on the promise's own executor. */
    @SuppressWarnings("unchecked")
    static void complete(Object promise, int kind, int status, long value, boolean[] replies) {
        Promise<Object> p = (Promise<Object>) promise;
        if (status != 0) {
            p.tryFailure(new org.redisson.client.RedisException("GPU call failed with status " + status));
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
    }
}
