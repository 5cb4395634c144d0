/*
 * RBitSet on the GPU keyspace: the object Redisson.getBitSet (Redisson.java:
 * 515-517) and RBatch.getBitSet (RedissonBatch.java:191) return when GPU
 * sketches are enabled.  The reference keeps a bit set as a Redis string
 * (MSB-first: bit i in byte i/8 under mask 0x80 >> i%8, RedissonBitSet.java:
 * 152-173) and a Bloom filter's bits ARE such a string under the filter's
 * name, so getBitSet(filterName) reads the bits RBloomFilter.add set: here the
 * name resolves in the context's keyspace to a plain string, or to the bits of
 * the GPU Bloom filter of that name (rsk_bloom_bitset: toByteArray returns the
 * bytes Redis's GET would, cardinality its BITCOUNT), or to nothing (an empty
 * string: toByteArray null, cardinality / length / size 0).
 *
 * Commands (RedissonBitSet.java): GETBIT / SETBIT (:53-81), GET (:88-91),
 * BITCOUNT (:240-243), STRLEN via BITS_SIZE (:230-233), the length() script
 * (:180-192), the set/clear(from, to) SETBIT loops as one range call
 * (:194-228), SET (:211-214), DEL (:250-253), BITOP op name name others
 * (:138-145, :216-268).  Every call runs on the GPU through the shim; the
 * futures are complete when the call returns (the library is synchronous for
 * these), so the inherited synchronous methods (get(xxxAsync())) and
 * asBitSet / toString work unchanged.  A name holding a GPU HyperLogLog is
 * refused (WRONGTYPE); expire / move / migrate fail as for the other GPU
 * objects (no TTL in GPU memory).
 */
package org.redisson.gpu;

import java.util.BitSet;
import java.util.Date;
import java.util.concurrent.TimeUnit;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

import org.redisson.RedissonBitSet;
import org.redisson.command.CommandAsyncExecutor;

public class GpuBitSet extends RedissonBitSet {

    private final GpuSketchContext gpu;

    public GpuBitSet(CommandAsyncExecutor commandExecutor, String name, GpuSketchContext gpu) {
        super(commandExecutor, name);
        this.gpu = gpu;
    }

    /* One synchronous native call as a completed future. */
    abstract static class Call<T> {
        abstract T run();
    }

    static <T> Future<T> now(GpuSketchContext gpu, Call<T> c) {
        Promise<T> p = gpu.newPromise();
        try {
            p.setSuccess(c.run());
        } catch (RuntimeException e) {
            p.tryFailure(e);
        }
        return p;
    }

    /* java.util.BitSet -> the SET bytes, as the reference encodes them:
     * bits.length() / 8 + 1 bytes, MSB-first within a byte (:163-173). */
    static byte[] encode(BitSet bits) {
        byte[] out = new byte[bits.length() / 8 + 1];
        for (int i = bits.nextSetBit(0); i >= 0; i = bits.nextSetBit(i + 1)) {
            out[i >>> 3] |= (byte) (0x80 >>> (i & 7));
        }
        return out;
    }

    private Future<Void> op(final int op, final String... others) {
        final String name = getName();
        return now(gpu, new Call<Void>() {
            Void run() {
                RSketchNative.bitsetOp(gpu.space, name, op, others);
                return null;
            }
        });
    }

    @Override
    public Future<byte[]> toByteArrayAsync() {
        final String name = getName();
        return now(gpu, new Call<byte[]>() {
            byte[] run() {
                return RSketchNative.bitsetGet(gpu.space, name);
            }
        });
    }

    @Override
    public Future<Long> lengthAsync() {
        final String name = getName();
        return now(gpu, new Call<Long>() {
            Long run() {
                return Long.valueOf(RSketchNative.bitsetLength(gpu.space, name));
            }
        });
    }

    @Override
    public Future<Void> setAsync(final long fromIndex, final long toIndex, final boolean value) {
        final String name = getName();
        return now(gpu, new Call<Void>() {
            Void run() {
                RSketchNative.bitsetSetRange(gpu.space, name, fromIndex, toIndex, value);
                return null;
            }
        });
    }

    @Override
    public Future<Void> clearAsync(long fromIndex, long toIndex) {
        return setAsync(fromIndex, toIndex, false);
    }

    @Override
    public Future<Void> setAsync(long fromIndex, long toIndex) {
        return setAsync(fromIndex, toIndex, true);
    }

    @Override
    public Future<Void> setAsync(BitSet bs) {
        final String name = getName();
        final byte[] bytes = encode(bs);
        return now(gpu, new Call<Void>() {
            Void run() {
                RSketchNative.bitsetSet(gpu.space, name, bytes);
                return null;
            }
        });
    }

    @Override
    public Future<Void> notAsync() {
        return op(RSketchNative.BITOP_NOT);
    }

    @Override
    public Future<Integer> sizeAsync() {
        final String name = getName();
        return now(gpu, new Call<Integer>() {
            Integer run() {  // BitsSizeReplayConvertor: STRLEN * 8 as an int
                return Integer.valueOf((int) (RSketchNative.bitsetStrlen(gpu.space, name) * 8));
            }
        });
    }

    @Override
    public Future<Boolean> getAsync(final long bitIndex) {
        final String name = getName();
        return now(gpu, new Call<Boolean>() {
            Boolean run() {
                return Boolean.valueOf(RSketchNative.bitsetGetBits(gpu.space, name, new long[] {bitIndex})[0]);
            }
        });
    }

    @Override
    public Future<Void> setAsync(long bitIndex) {
        return setAsync(bitIndex, true);
    }

    @Override
    public Future<Void> setAsync(final long bitIndex, final boolean value) {
        final String name = getName();
        return now(gpu, new Call<Void>() {
            Void run() {
                RSketchNative.bitsetSetBits(gpu.space, name, new long[] {bitIndex}, value);
                return null;
            }
        });
    }

    @Override
    public Future<Long> cardinalityAsync() {
        final String name = getName();
        return now(gpu, new Call<Long>() {
            Long run() {
                return Long.valueOf(RSketchNative.bitsetCardinality(gpu.space, name));
            }
        });
    }

    @Override
    public Future<Void> clearAsync(long bitIndex) {
        return setAsync(bitIndex, false);
    }

    @Override
    public Future<Void> clearAsync() {
        final String name = getName();
        return now(gpu, new Call<Void>() {
            Void run() {
                RSketchNative.bitsetClear(gpu.space, name);
                return null;
            }
        });
    }

    @Override
    public Future<Void> orAsync(String... bitSetNames) {
        return op(RSketchNative.BITOP_OR, bitSetNames);
    }

    @Override
    public Future<Void> andAsync(String... bitSetNames) {
        return op(RSketchNative.BITOP_AND, bitSetNames);
    }

    @Override
    public Future<Void> xorAsync(String... bitSetNames) {
        return op(RSketchNative.BITOP_XOR, bitSetNames);
    }

    /* Batched GETBIT / SETBIT over many indexes: one native call. */
    public boolean[] getBits(long[] indexes) {
        return RSketchNative.bitsetGetBits(gpu.space, getName(), indexes);
    }

    public void setBits(long[] indexes, boolean value) {
        RSketchNative.bitsetSetBits(gpu.space, getName(), indexes, value);
    }

    // ---------------------------------------------------------------- keyspace
    @Override
    public Future<Boolean> deleteAsync() {  // DEL name: the string (a filter's config stays)
        final String name = getName();
        return now(gpu, new Call<Boolean>() {
            Boolean run() {
                return Boolean.valueOf(RSketchNative.bitsetClear(gpu.space, name));
            }
        });
    }

    @Override
    public Future<Boolean> isExistsAsync() {
        final String name = getName();
        return now(gpu, new Call<Boolean>() {
            Boolean run() {
                return Boolean.valueOf(RSketchNative.bitsetStrlen(gpu.space, name) > 0);
            }
        });
    }

    @Override
    public Future<Void> renameAsync(final String newName) {
        final String name = getName();
        return now(gpu, new Call<Void>() {
            Void run() {
                GpuKeyspace.rename(gpu, name, newName, false);
                return null;
            }
        });
    }

    @Override
    public Future<Boolean> renamenxAsync(final String newName) {
        final String name = getName();
        return now(gpu, new Call<Boolean>() {
            Boolean run() {
                return Boolean.valueOf(GpuKeyspace.rename(gpu, name, newName, true));
            }
        });
    }

    @Override
    public Future<Boolean> expireAsync(long timeToLive, TimeUnit timeUnit) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> expireAtAsync(long timestamp) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> expireAtAsync(Date timestamp) {
        return gpu.failed(GpuKeyspace.noTtl());
    }

    @Override
    public Future<Boolean> clearExpireAsync() {
        Promise<Boolean> p = gpu.newPromise();
        p.setSuccess(Boolean.FALSE);
        return p;
    }

    @Override
    public Future<Long> remainTimeToLiveAsync() {
        Promise<Long> p = gpu.newPromise();
        p.setSuccess(Long.valueOf(-1));
        return p;
    }

    @Override
    public Future<Boolean> moveAsync(int database) {
        return gpu.failed(GpuKeyspace.notOnGpu("move"));
    }

    @Override
    public Future<Void> migrateAsync(String host, int port, int database) {
        return gpu.failed(GpuKeyspace.notOnGpu("migrate"));
    }
}
