"""Element -> bytes codecs: which bytes get hashed.

Mirrors the reference's value encoders:
  * JsonJacksonCodec (default, src/main/java/org/redisson/Config.java:68-70;
    src/main/java/org/redisson/codec/JsonJacksonCodec.java:56-117):
    String "foo" -> b'"foo"', Integer 1 -> b'1', Long v -> b'["java.lang.Long",v]'
    (Long is force-typed, JsonJacksonCodec.java:104-106; Jackson writes the
    type id of a scalar as a wrapper array).
  * StringCodec / LongCodec: UTF-8 of toString() (client/codec/StringCodec.java).
  * ByteArrayCodec: bytes unchanged (client/codec/ByteArrayCodec.java:30-34).

Host-side only: keys reach the GPU already encoded.
"""
from __future__ import annotations


class JavaLong(int):
    """A Python int that the reference would hold as java.lang.Long."""


class JavaInteger(int):
    """A Python int that the reference would hold as java.lang.Integer."""


_JSON_SHORT = {0x08: "\\b", 0x09: "\\t", 0x0A: "\\n", 0x0C: "\\f", 0x0D: "\\r", 0x22: '\\"', 0x5C: "\\\\"}


def _json_string(s: str) -> str:
    out = []
    for ch in s:
        o = ord(ch)
        if o in _JSON_SHORT:
            out.append(_JSON_SHORT[o])
        elif o < 0x20:
            out.append("\\u%04X" % o)
        else:
            out.append(ch)
    return '"' + "".join(out) + '"'


class Codec:
    name = "codec"

    def encode(self, obj) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError


class JsonJacksonCodec(Codec):
    """Jackson ObjectMapper output for the scalar types sketches are fed."""

    name = "JsonJacksonCodec"

    def encode(self, obj) -> bytes:
        if isinstance(obj, bool):
            return b"true" if obj else b"false"
        if isinstance(obj, JavaLong):
            return ('["java.lang.Long",%d]' % int(obj)).encode()
        if isinstance(obj, int):
            # A bare Python int is an Integer when it fits, else a Long.
            if -(1 << 31) <= obj < (1 << 31) and not isinstance(obj, JavaLong):
                return str(int(obj)).encode()
            return ('["java.lang.Long",%d]' % int(obj)).encode()
        if isinstance(obj, str):
            return _json_string(obj).encode("utf-8")
        if isinstance(obj, (bytes, bytearray, memoryview)):
            import base64  # Jackson writes byte[] as a base64 JSON string

            return ('"%s"' % base64.b64encode(bytes(obj)).decode()).encode()
        raise TypeError("JsonJacksonCodec mirror supports str/int/bool/bytes; pre-encode %r with ByteArrayCodec"
                        % type(obj).__name__)


class StringCodec(Codec):
    name = "StringCodec"

    def encode(self, obj) -> bytes:
        if isinstance(obj, (bytes, bytearray)):
            return bytes(obj)
        if isinstance(obj, bool):
            return b"true" if obj else b"false"
        return str(obj).encode("utf-8")


class LongCodec(StringCodec):
    name = "LongCodec"


class ByteArrayCodec(Codec):
    name = "ByteArrayCodec"

    def encode(self, obj) -> bytes:
        if not isinstance(obj, (bytes, bytearray, memoryview)):
            raise TypeError("ByteArrayCodec takes bytes")
        return bytes(obj)


DEFAULT_CODEC = JsonJacksonCodec()
