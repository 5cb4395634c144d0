/*
 * Native methods of the GPU sketch engine (librsketch.so) as the JNI glue
 * jni/rsketch_jni.c exports them.  Handles are the C pointers as longs.
 * Key batches are direct buffers (GetDirectBufferAddress, no copy): the
 * codec-encoded elements back to back, and n+1 byte offsets in native order
 * (see KeyBuffer).  Errors arrive as the exceptions the Redis path raises
 * (IllegalArgumentException, IllegalStateException, RedisException).
 */
package org.redisson.gpu;

import java.nio.ByteBuffer;
import java.nio.LongBuffer;

final class RSketchNative {

    static {
        System.loadLibrary("rsketch_jni"); // links librsketch.so
    }

    private RSketchNative() {
    }

    static native long init(int device);                                  // rsk_init
    static native void shutdown(long ctx);                                // rsk_shutdown

    static native long hllCreate(long ctx, long nSketches);               // rsk_hll_create
    static native void hllDestroy(long hll);
    static native boolean hllAdd(long hll, long id, ByteBuffer keys, LongBuffer offsets, long n);        // PFADD id e1..en
    static native boolean[] hllAddEach(long hll, long id, ByteBuffer keys, LongBuffer offsets, long n);  // n x PFADD id e
    static native long hllCount(long hll, long id);                       // PFCOUNT id
    static native long hllCountUnion(long[] hlls, long[] ids);            // PFCOUNT k1..kk
    static native void hllMerge(long dst, long dstId, long[] srcs, long[] srcIds); // PFMERGE dst src..
    static native void hllDelete(long hll, long id);                      // DEL

    static native long[] bloomParams(long expectedInsertions, double falseProbability, boolean extended); // {size, k}
    static native long bloomCreate(long ctx, long size, int k);
    static native void bloomDestroy(long bloom);
    static native boolean[] bloomAdd(long bloom, ByteBuffer keys, LongBuffer offsets, long n);
    static native boolean[] bloomContains(long bloom, ByteBuffer keys, LongBuffer offsets, long n);
    static native int bloomCount(long bloom);
}
