/*
 * One batch of elements encoded with the object's codec, exactly the bytes the
 * Redis path would send (CommandEncoder.java:77-79: codec.getValueEncoder().encode(o);
 * RedissonBloomFilter.java:170-178), packed into direct buffers for one native call.
 */
package org.redisson.gpu;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.LongBuffer;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;

import org.redisson.client.codec.Codec;

final class KeyBuffer {

    final ByteBuffer bytes;
    final LongBuffer offsets;
    final long n;

    private KeyBuffer(ByteBuffer bytes, LongBuffer offsets, long n) {
        this.bytes = bytes;
        this.offsets = offsets;
        this.n = n;
    }

    /* One element's codec bytes (IllegalArgumentException on a codec failure, :170-178). */
    static byte[] encodeElement(Codec codec, Object o) {
        try {
            return codec.getValueEncoder().encode(o);
        } catch (IOException e) {
            throw new IllegalArgumentException(e);
        }
    }

    static KeyBuffer encode(Codec codec, Collection<?> objects) {
        List<byte[]> enc = new ArrayList<byte[]>(objects.size());
        for (Object o : objects) {
            enc.add(encodeElement(codec, o));
        }
        return ofEncoded(enc);
    }

    /* Elements already encoded (a batch queued element by element). */
    static KeyBuffer ofEncoded(List<byte[]> enc) {
        long total = 0;
        for (byte[] b : enc) {
            total += b.length;
        }
        if (total > Integer.MAX_VALUE) {
            throw new IllegalArgumentException("batch larger than 2 GiB: split it");
        }
        ByteBuffer data = ByteBuffer.allocateDirect((int) Math.max(1, total));
        ByteBuffer ob = ByteBuffer.allocateDirect(8 * (enc.size() + 1)).order(ByteOrder.nativeOrder());
        LongBuffer offs = ob.asLongBuffer();
        long pos = 0;
        offs.put(0, 0L);
        for (int i = 0; i < enc.size(); i++) {
            byte[] b = enc.get(i);
            data.put(b);
            pos += b.length;
            offs.put(i + 1, pos);
        }
        data.clear();
        return new KeyBuffer(data, offs, enc.size());
    }

    static KeyBuffer encodeOne(Codec codec, Object o) {
        List<Object> one = new ArrayList<Object>(1);
        one.add(o);
        return encode(codec, one);
    }
}
