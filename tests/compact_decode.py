"""Schema-less Thrift Compact protocol decoder (test infrastructure).

Written from the Apache Thrift Compact protocol specification, independently
of the product's C++ codec (openr_amd/csrc/host/thrift_compact.cpp): a struct
decodes to {field id: value}, lists and sets to Python lists, maps to dicts,
binary to bytes, integers to int, bools to bool. Tests decode the product's
bytes with it and compare against the route databases they describe.
"""

STOP, TRUE, FALSE, BYTE, I16, I32, I64, DOUBLE, BINARY, LIST, SET, MAP, STRUCT = range(13)


class Decoder:
    def __init__(self, data: bytes):
        self.b = data
        self.i = 0

    def byte(self):
        v = self.b[self.i]
        self.i += 1
        return v

    def varint(self):
        shift = v = 0
        while True:
            c = self.byte()
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7

    def zigzag(self):
        u = self.varint()
        return (u >> 1) ^ -(u & 1)

    def value(self, t):
        if t in (TRUE, FALSE):  # list element: one byte
            return self.byte() == TRUE
        if t == BYTE:
            return self.byte()
        if t in (I16, I32, I64):
            return self.zigzag()
        if t == DOUBLE:
            raise ValueError("double not used on this path")
        if t == BINARY:
            n = self.varint()
            v = self.b[self.i:self.i + n]
            self.i += n
            return bytes(v)
        if t in (LIST, SET):
            h = self.byte()
            n, et = h >> 4, h & 0x0F
            if n == 15:
                n = self.varint()
            return [self.value(et) for _ in range(n)]
        if t == MAP:
            n = self.varint()
            if n == 0:
                return {}
            kv = self.byte()
            out = {}
            for _ in range(n):
                k = self.value(kv >> 4)
                out[k if not isinstance(k, list) else tuple(k)] = self.value(kv & 0x0F)
            return out
        if t == STRUCT:
            return self.struct()
        raise ValueError(f"unknown type {t}")

    def struct(self):
        out, last = {}, 0
        while True:
            h = self.byte()
            if h == STOP:
                return out
            t, d = h & 0x0F, h >> 4
            fid = last + d if d else self.zigzag()
            last = fid
            out[fid] = (t == TRUE) if t in (TRUE, FALSE) else self.value(t)


def decode(data: bytes):
    d = Decoder(data)
    v = d.struct()
    if d.i != len(data):
        raise ValueError("trailing bytes")
    return v
