/*
 * RBloomFilter on the GPU (Redisson.getBloomFilter, Redisson.java:525-532).
 * Same sizing (optimalNumOfBits / optimalNumOfHashFunctions, MAX_SIZE,
 * RedissonBloomFilter.java:52,69-78,223-229), same hash scheme (xx_r39 +
 * farmUo, (h & Long.MAX_VALUE) % size, :116-131), same replies: add() is true
 * iff one of the first k-1 SETBITs found its bit clear (:100-107), contains()
 * is the AND of the first k-1 GETBITs (:147-168), count() the BITCOUNT
 * formula (:188-199).  tryInit creates the filter; the {name}__config hash
 * keeps its fields for wire interop (redisson_amd/bloom.py mirrors it).
 */
package org.redisson.gpu;

import java.util.Collection;
import java.util.concurrent.Callable;

import org.redisson.RedissonBloomFilter;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandExecutor;

public class GpuBloomFilter<T> extends RedissonBloomFilter<T> {

    private final GpuSketchContext gpu;
    private final Codec valueCodec;
    private final boolean extended;
    private volatile long size;
    private volatile int hashIterations;
    private volatile long expectedInsertions;
    private volatile double falseProbability;

    public GpuBloomFilter(Codec codec, CommandExecutor commandExecutor, String name, GpuSketchContext gpu,
                          boolean extended) {
        super(codec, commandExecutor, name);
        this.valueCodec = codec;
        this.gpu = gpu;
        this.extended = extended;
    }

    private long handle() {
        Long b = gpu.bloom(getName());
        if (b == null) {
            throw new IllegalStateException("Bloom filter is not initialized!");
        }
        return b;
    }

    @Override
    public boolean tryInit(final long expectedInsertions, final double falseProbability) {
        return gpu.call(new Callable<Boolean>() {
            public Boolean call() {
                if (gpu.bloom(getName()) != null) {
                    return false;
                }
                long[] p = RSketchNative.bloomParams(expectedInsertions, falseProbability, extended);
                gpu.putBloom(getName(), RSketchNative.bloomCreate(gpu.ctx, p[0], (int) p[1]));
                GpuBloomFilter.this.size = p[0];
                GpuBloomFilter.this.hashIterations = (int) p[1];
                GpuBloomFilter.this.expectedInsertions = expectedInsertions;
                GpuBloomFilter.this.falseProbability = falseProbability;
                return true;
            }
        });
    }

    /* One native call for a whole batch (the Redis path: k SETBITs per element). */
    public boolean[] addAll(final Collection<T> objects) {
        return gpu.call(new Callable<boolean[]>() {
            public boolean[] call() {
                KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
                return RSketchNative.bloomAdd(handle(), kb.bytes, kb.offsets, kb.n);
            }
        });
    }

    public boolean[] containsAll(final Collection<T> objects) {
        return gpu.call(new Callable<boolean[]>() {
            public boolean[] call() {
                KeyBuffer kb = KeyBuffer.encode(valueCodec, objects);
                return RSketchNative.bloomContains(handle(), kb.bytes, kb.offsets, kb.n);
            }
        });
    }

    @Override
    public boolean add(final T object) {
        return gpu.call(new Callable<Boolean>() {
            public Boolean call() {
                KeyBuffer kb = KeyBuffer.encodeOne(valueCodec, object);
                return RSketchNative.bloomAdd(handle(), kb.bytes, kb.offsets, 1)[0];
            }
        });
    }

    @Override
    public boolean contains(final T object) {
        return gpu.call(new Callable<Boolean>() {
            public Boolean call() {
                KeyBuffer kb = KeyBuffer.encodeOne(valueCodec, object);
                return RSketchNative.bloomContains(handle(), kb.bytes, kb.offsets, 1)[0];
            }
        });
    }

    @Override
    public int count() {
        return gpu.call(new Callable<Integer>() {
            public Integer call() {
                return RSketchNative.bloomCount(handle());
            }
        });
    }

    @Override
    public long getSize() {
        return size;
    }

    @Override
    public int getHashIterations() {
        return hashIterations;
    }

    @Override
    public long getExpectedInsertions() {
        return expectedInsertions;
    }

    @Override
    public double getFalseProbability() {
        return falseProbability;
    }

    @Override
    public boolean delete() {
        return gpu.call(new Callable<Boolean>() {
            public Boolean call() {
                return gpu.dropBloom(getName());
            }
        });
    }
}
