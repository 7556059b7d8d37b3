"""Hand-built Binary/Compact wire bytes for semantic and malformed-input tests
(independent of both the oracle and the device writers)."""
import struct

B, C = 0, 2  # protocol ids

# Compact types (CompactProtocol-inl.h:31-46)
CT = {2: 1, 3: 3, 6: 4, 8: 5, 10: 6, 4: 7, 11: 8, 15: 9, 14: 10, 13: 11, 12: 12, 19: 13}


def varint(v):
    out = bytearray()
    while v & ~0x7F:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def zz32(n):
    return ((n << 1) ^ (n >> 31)) & 0xFFFFFFFF


def zz64(n):
    return ((n << 1) ^ (n >> 63)) & 0xFFFFFFFFFFFFFFFF


class W:
    """Minimal writer following the reference's wire rules."""

    def __init__(self, proto):
        self.p, self.b, self.last = proto, bytearray(), [0]

    def field(self, ttype, fid, bool_value=None):
        if self.p == B:
            self.b += bytes([ttype]) + struct.pack(">h", fid)
        else:
            ct = CT[ttype]
            if ttype == 2:
                ct = 1 if bool_value else 2
            d = fid - self.last[-1]
            if 0 < d <= 15:
                self.b.append((d << 4) | ct)
            else:
                self.b.append(ct)
                self.b += varint(zz32(fid))
            self.last[-1] = fid
        return self

    def stop(self):
        self.b.append(0)
        return self

    def struct_begin(self):
        self.last.append(0)
        return self

    def struct_end(self):
        self.stop()
        self.last.pop()
        return self

    def i32(self, v):
        self.b += struct.pack(">i", v) if self.p == B else varint(zz32(v))
        return self

    def i64(self, v):
        self.b += struct.pack(">q", v) if self.p == B else varint(zz64(v))
        return self

    def byte(self, v):
        self.b.append(v & 0xFF)
        return self

    def string(self, s):
        self.b += (struct.pack(">i", len(s)) if self.p == B else varint(len(s))) + s
        return self

    def list_begin(self, etype, n):
        if self.p == B:
            self.b += bytes([etype]) + struct.pack(">i", n)
        elif n <= 14:
            self.b.append((n << 4) | CT[etype])
        else:
            self.b.append(0xF0 | CT[etype])
            self.b += varint(n)
        return self

    def map_begin(self, kt, vt, n):
        if self.p == B:
            self.b += bytes([kt, vt]) + struct.pack(">i", n)
        elif n == 0:
            self.b.append(0)
        else:
            self.b += varint(n) + bytes([(CT[kt] << 4) | CT[vt]])
        return self

    def raw(self, bs):
        self.b += bs
        return self

    def bytes(self):
        return bytes(self.b)


def nested(proto, height, levels, ttype):
    """ProtocolTest.cpp:170-259 makeNested(): a struct holding `height` fields
    nested (levels - 3) deep plus one nested (levels - 2) deep (field id 0)."""
    w = W(proto)

    def inner(lv):
        if ttype == 12:
            for _ in range(lv):
                w.struct_begin().field(12, 0)
            w.struct_begin().field(3, 0).byte(7).struct_end()
            for _ in range(lv):
                w.struct_end()
        elif ttype in (15, 14):
            for _ in range(lv):
                w.list_begin(ttype, 1)
            w.list_begin(3, 1).byte(7)
        elif ttype == 13:
            for _ in range(lv):
                w.map_begin(3, 13, 1).byte(7)
            w.map_begin(3, 3, 1).byte(7).byte(7)

    for _ in range(height):
        w.field(ttype, 0)
        inner(levels - 3)
    w.field(ttype, 0)
    inner(levels - 2)
    w.stop()
    return w.bytes()
