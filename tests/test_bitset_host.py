"""Host-side java.util.BitSet conversions of RedissonBitSet (CPU only)."""
from redisson_amd.bitset import JavaBitSet, from_byte_array_reverse, to_byte_array_reverse


def test_msb_first_roundtrip():
    bs = JavaBitSet([1, 10])
    data = to_byte_array_reverse(bs)
    assert data == bytes([0b01000000, 0b00100000])  # length()/8 + 1 = 2 bytes
    assert from_byte_array_reverse(data) == bs
    assert str(bs) == "{1, 10}"


def test_to_byte_array_reverse_extra_byte():
    # RedissonBitSet.toByteArrayReverse allocates length()/8 + 1 bytes even when
    # length() is a multiple of 8 (BitSet{7} -> 2 bytes, so size() becomes 16).
    assert to_byte_array_reverse(JavaBitSet([7])) == bytes([0b00000001, 0])
    assert to_byte_array_reverse(JavaBitSet()) == b"\x00"


def test_from_bytes_all_bits():
    assert from_byte_array_reverse(b"\xff").indices() == list(range(8))
    assert from_byte_array_reverse(b"").cardinality() == 0
