"""Host-side codecs decide which bytes are hashed (CommandEncoder.java:77-79)."""
from redisson_amd.codec import ByteArrayCodec, JavaLong, JsonJacksonCodec, LongCodec, StringCodec
from redisson_amd.keys import KeyBatch


def test_json_scalars():
    c = JsonJacksonCodec()
    assert c.encode(1) == b"1"                      # Integer (RedissonHyperLogLogTest.testAdd)
    assert c.encode("foo") == b'"foo"'              # String (testMerge)
    assert c.encode(JavaLong(123)) == b'["java.lang.Long",123]'
    assert c.encode(1 << 40) == b'["java.lang.Long",1099511627776]'
    assert c.encode(True) == b"true"
    assert c.encode('a"b\\c\n') == b'"a\\"b\\\\c\\n"'
    assert c.encode("\x01") == b'"\\u0001"'
    assert c.encode("é") == '"é"'.encode()


def test_string_long_bytearray():
    assert StringCodec().encode(123) == b"123"
    assert LongCodec().encode(-5) == b"-5"
    assert ByteArrayCodec().encode(b"\x00\xff") == b"\x00\xff"


def test_keybatch_fixed_and_var():
    kb = KeyBatch.from_bytes_list([b"ab", b"cd", b"ef"])
    assert kb.fixed_len == 2 and kb.offsets is None and kb.n == 3
    kb = KeyBatch.from_bytes_list([b"a", b"", b"xyz"])
    assert kb.fixed_len == 0 and kb.offsets is not None and kb.n == 3
    s = kb.slice(1, 3)
    assert s.n == 2
