/*
 * One GPU (one rsk_ctx) and its keyspace (jni/rsketch_shim.h): the objects
 * below address their sketches by NAME, as the Redis-backed objects address
 * keys, so two instances with one name share one sketch, a second
 * getBloomFilter(name) sees the size and k the first one initialised, and
 * count() of a name nobody wrote creates nothing.  There is no executor thread:
 * synchronous calls go straight to the library (which orders every call of a
 * context on one HIP stream), asynchronous ones return a Netty promise that
 * the library's completion callback fulfils (RSketchNative.complete), the way
 * a Redis reply completes CommandAsyncService's promise (:86-105).
 */
package org.redisson.gpu;

import io.netty.util.concurrent.Promise;

import org.redisson.connection.ConnectionManager;

public final class GpuSketchContext {

    final long space;
    private final ConnectionManager connectionManager;

    /* extendedBloom: tryInit may size filters above RedissonBloomFilter.MAX_SIZE
     * (the reference throws IllegalArgumentException there, :226-227). */
    public GpuSketchContext(ConnectionManager connectionManager, int device, boolean extendedBloom) {
        this.connectionManager = connectionManager;
        this.space = RSketchNative.init(device, extendedBloom);
    }

    public GpuSketchContext(ConnectionManager connectionManager, int device) {
        this(connectionManager, device, false);
    }

    <T> Promise<T> newPromise() {
        return connectionManager.newPromise();
    }

    /* A promise that failed at once (the call was refused before it started). */
    <T> Promise<T> failed(Throwable t) {
        Promise<T> p = connectionManager.newPromise();
        p.setFailure(t);
        return p;
    }

    /* TYPE-like probe: RSketchNative.NONE / HLL / BLOOM. */
    public int type(String name) {
        return RSketchNative.type(space, name);
    }

    public boolean delete(String name) {
        return RSketchNative.delete(space, name);
    }

    public GpuBatch createBatch() {
        return new GpuBatch(this);
    }

    public void shutdown() {
        RSketchNative.shutdown(space);
    }
}
