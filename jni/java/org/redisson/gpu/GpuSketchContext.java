/*
 * One GPU (one rsk_ctx) and the sketches living on it.  A name maps to a
 * (pool, id) slot so countWith/mergeWith resolve other names the way Redis
 * resolves keys; every native call of one context runs on its single
 * executor thread (the library serialises a context on one HIP stream
 * anyway), which is also where the async variants complete their promises.
 */
package org.redisson.gpu;

import java.util.HashMap;
import java.util.Map;
import java.util.concurrent.Callable;
import java.util.concurrent.ExecutionException;
import java.util.concurrent.ExecutorService;
import java.util.concurrent.Executors;
import java.util.concurrent.ThreadFactory;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

import org.redisson.connection.ConnectionManager;

public final class GpuSketchContext {

    final long ctx;
    private final ExecutorService gpu;
    private final ConnectionManager connectionManager;
    private final Map<String, Long> hlls = new HashMap<String, Long>();
    private final Map<String, Long> blooms = new HashMap<String, Long>();

    public GpuSketchContext(ConnectionManager connectionManager, int device) {
        this.connectionManager = connectionManager;
        this.ctx = RSketchNative.init(device);
        this.gpu = Executors.newSingleThreadExecutor(new ThreadFactory() {
            public Thread newThread(Runnable r) {
                Thread t = new Thread(r, "redisson-gpu-sketch");
                t.setDaemon(true);
                return t;
            }
        });
    }

    /* The HLL slot of `name` (a one-sketch pool per key). */
    synchronized long hll(String name) {
        Long h = hlls.get(name);
        if (h == null) {
            h = RSketchNative.hllCreate(ctx, 1);
            hlls.put(name, h);
        }
        return h;
    }

    synchronized Long bloom(String name) {
        return blooms.get(name);
    }

    synchronized void putBloom(String name, long b) {
        blooms.put(name, b);
    }

    synchronized boolean dropBloom(String name) {
        Long b = blooms.remove(name);
        if (b != null) {
            RSketchNative.bloomDestroy(b);
        }
        return b != null;
    }

    <T> T call(Callable<T> c) {
        try {
            return gpu.submit(c).get();
        } catch (InterruptedException e) {
            Thread.currentThread().interrupt();
            throw new IllegalStateException(e);
        } catch (ExecutionException e) {
            Throwable t = e.getCause();
            if (t instanceof RuntimeException) {
                throw (RuntimeException) t;
            }
            throw new IllegalStateException(t);
        }
    }

    <T> Future<T> callAsync(final Callable<T> c) {
        final Promise<T> p = connectionManager.newPromise();
        gpu.execute(new Runnable() {
            public void run() {
                try {
                    p.setSuccess(c.call());
                } catch (Throwable t) {
                    p.setFailure(t);
                }
            }
        });
        return p;
    }

    public synchronized void shutdown() {
        gpu.shutdown();
        for (Long h : hlls.values()) {
            RSketchNative.hllDestroy(h);
        }
        for (Long b : blooms.values()) {
            RSketchNative.bloomDestroy(b);
        }
        hlls.clear();
        blooms.clear();
        RSketchNative.shutdown(ctx);
    }
}
