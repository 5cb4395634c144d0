/*
 * The reactive mirrors' one adapter: a GPU call's future as the Publisher
 * the reference's reactive objects return.  RedissonObjectReactive.reactive
 * (src/main/java/org/redisson/reactive/RedissonObjectReactive.java:41-43)
 * hands a Redis reply's future to CommandReactiveService.reactive, which wraps
 * it in a NettyFuturePublisher (reactive/NettyFuturePublisher.java:27-70: on
 * request, one onNext with the value unless it is null, then onComplete;
 * onError on failure).  The GPU objects' futures are completed by the
 * library's completion (on the context's event loop) or at once, so the same
 * publisher serves them unchanged.
 */
package org.redisson.gpu;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.FutureListener;
import io.netty.util.concurrent.Promise;

import org.reactivestreams.Publisher;
import org.redisson.reactive.NettyFuturePublisher;

final class GpuReactive {

    private GpuReactive() {
    }

    static <R> Publisher<R> publisher(Future<R> future) {
        return new NettyFuturePublisher<R>(future);
    }

    /* A value derived from a future's value (null stays null: nothing is emitted). */
    abstract static class Map<A, B> {
        abstract B apply(A a);
    }

    static <A, B> Future<B> map(GpuSketchContext gpu, Future<A> in, final Map<A, B> f) {
        final Promise<B> out = gpu.newPromise();
        in.addListener(new FutureListener<A>() {
            @Override
            public void operationComplete(Future<A> done) {
                if (!done.isSuccess()) {
                    out.tryFailure(done.cause());
                    return;
                }
                try {
                    A a = done.getNow();
                    out.trySuccess(a == null ? null : f.apply(a));
                } catch (RuntimeException e) {
                    out.tryFailure(e);
                }
            }
        });
        return out;
    }
}
