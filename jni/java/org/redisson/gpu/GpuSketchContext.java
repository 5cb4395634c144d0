/*
 * One GPU (one rsk_ctx) and its keyspace (jni/rsketch_shim.h): the objects
 * below address their sketches by NAME, as the Redis-backed objects address
 * keys, so two instances with one name share one sketch, a second
 * getBloomFilter(name) sees the size and k the first one initialised,
 * getBitSet(name) of a Bloom filter's name reads its bits, and count() of a
 * name nobody wrote creates nothing.  There is no executor thread for calls:
 * synchronous calls go straight to the library (which orders every call of a
 * context on one HIP stream), asynchronous ones return a Netty promise that
 * the library's completion fulfils.
 *
 * Where listeners run.  The reference's promises come from
 * connectionManager.newPromise(), i.e. ImmediateEventExecutor
 * (MasterSlaveConnectionManager.java:680-682): listeners run on whatever thread
 * completes the promise, which for a Redis reply is the connection's Netty
 * event loop.  Here the library's completion thread must not be that thread
 * (a listener would run inside the library's callback), so every completion
 * is handed to ONE event loop of the connection manager's group, pinned per
 * context: listeners run on a Netty event loop, as for a Redis reply, and in
 * the order the calls were issued (the library delivers completions in
 * submission order; one loop keeps that order).
 */
package org.redisson.gpu;

import io.netty.channel.EventLoop;
import io.netty.util.concurrent.Promise;

import org.redisson.connection.ConnectionManager;

public final class GpuSketchContext {

    final long space;
    private final ConnectionManager connectionManager;
    private final EventLoop completions;

    /* extendedBloom: tryInit may size filters above RedissonBloomFilter.MAX_SIZE
     * (the reference throws IllegalArgumentException there, :226-227). */
    public GpuSketchContext(ConnectionManager connectionManager, int device, boolean extendedBloom) {
        this.connectionManager = connectionManager;
        this.completions = connectionManager.getGroup().next();
        this.space = RSketchNative.init(device, extendedBloom);
    }

    public GpuSketchContext(ConnectionManager connectionManager, int device) {
        this(connectionManager, device, false);
    }

    <T> Promise<T> newPromise() {
        return connectionManager.newPromise();
    }

    /* The completion an asynchronous native call fulfils: the promise, and the
     * event loop its listeners run on. */
    <T> RSketchNative.Completion<T> completion(Promise<T> p) {
        return new RSketchNative.Completion<T>(p, completions);
    }

    /* A promise that failed at once (the call was refused before it started). */
    <T> Promise<T> failed(Throwable t) {
        Promise<T> p = connectionManager.newPromise();
        p.setFailure(t);
        return p;
    }

    /* TYPE-like probe: RSketchNative.NONE / HLL / BLOOM / BITSET. */
    public int type(String name) {
        return RSketchNative.type(space, name);
    }

    public boolean delete(String name) {
        return RSketchNative.delete(space, name);
    }

    public GpuBatch createBatch() {
        return new GpuBatch(this);
    }

    /* Every call issued so far has completed and its completion is queued on
     * the event loop. */
    public void sync() {
        RSketchNative.sync(space);
    }

    /* Releases the context even when it is dead (a device error: sync() then
     * throws, and every later call fails): the native shutdown always runs. */
    public void shutdown() {
        try {
            RSketchNative.sync(space);
        } finally {
            RSketchNative.shutdown(space);
        }
    }
}
