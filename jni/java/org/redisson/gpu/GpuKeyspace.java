/*
 * Keyspace operations the GPU objects share (RedissonObject.java:72-130,
 * RedissonExpirable.java:40-88): the sketch lives in GPU memory, so the calls
 * that would act on a Redis key act on the context's keyspace, and the ones
 * that cannot be honoured there fail loudly instead of being dropped.
 */
package org.redisson.gpu;

final class GpuKeyspace {

    private GpuKeyspace() {
    }

    /* RENAME / RENAMENX old new on the GPU keyspace (rsk_shim_rename). */
    static boolean rename(GpuSketchContext gpu, String oldName, String newName, boolean nx) {
        return RSketchNative.rename(gpu.space, oldName, newName, nx);
    }

    static UnsupportedOperationException noTtl() {
        return new UnsupportedOperationException(
                "expire is not supported for GPU-resident sketches: the key lives in GPU memory, not in Redis");
    }

    static UnsupportedOperationException notOnGpu(String op) {
        return new UnsupportedOperationException(op + " is not supported for GPU-resident sketches");
    }
}
