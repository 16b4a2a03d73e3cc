"""Debug aid: dump the structs and delete set of a V1 update (test infrastructure, not the product path).
Usage: python tools/ydump.py <b64 or file>  -- or import dump_v1(bytes) -> list of lines."""
import base64
import struct
import sys


class R:
    def __init__(self, b):
        self.b, self.p = b, 0

    def u8(self):
        v = self.b[self.p]
        self.p += 1
        return v

    def vu(self):
        r, s = 0, 0
        while True:
            x = self.u8()
            r |= (x & 0x7F) << s
            s += 7
            if x < 0x80:
                return r

    def vi(self):
        x = self.u8()
        neg, r, s = x & 0x40, x & 0x3F, 6
        while x & 0x80:
            x = self.u8()
            r |= (x & 0x7F) << s
            s += 7
        return -r if neg else r

    def buf(self):
        n = self.vu()
        v = self.b[self.p:self.p + n]
        self.p += n
        return bytes(v)

    def s(self):
        return self.buf().decode("utf-8", "surrogatepass")

    def any(self):
        t = self.u8()
        if t == 127: return "undefined"
        if t == 126: return None
        if t == 125: return self.vi()
        if t == 124:
            v = struct.unpack(">f", self.b[self.p:self.p + 4])[0]; self.p += 4; return v
        if t == 123:
            v = struct.unpack(">d", self.b[self.p:self.p + 8])[0]; self.p += 8; return v
        if t == 122:
            v = struct.unpack(">q", self.b[self.p:self.p + 8])[0]; self.p += 8; return f"{v}n"
        if t == 121: return False
        if t == 120: return True
        if t == 119: return self.s()
        if t == 118:
            return {self.s(): self.any() for _ in range(self.vu())}
        if t == 117:
            return [self.any() for _ in range(self.vu())]
        if t == 116: return self.buf()
        raise ValueError(f"any tag {t}")


def dump_v1(b):
    r, out = R(b), []
    for _ in range(r.vu()):
        n, client, clock = r.vu(), r.vu(), r.vu()
        out.append(f"client {client} from {clock}: {n} structs")
        for _ in range(n):
            info = r.u8()
            ref = info & 31
            if ref == 0 or ref == 10:
                ln = r.vu()
                out.append(f"  {client}:{clock} {'GC' if ref == 0 else 'Skip'} len {ln}")
                clock += ln
                continue
            o = (r.vu(), r.vu()) if info & 0x80 else None
            ro = (r.vu(), r.vu()) if info & 0x40 else None
            par = sub = None
            if not (info & 0xC0):
                par = ("key", r.s()) if r.vu() == 1 else ("id", r.vu(), r.vu())
                if info & 0x20:
                    sub = r.s()
            if ref == 1: c = ("Deleted", r.vu()); ln = c[1]
            elif ref == 2: c = ("JSON", [r.s() for _ in range(r.vu())]); ln = len(c[1])
            elif ref == 3: c = ("Binary", r.buf()); ln = 1
            elif ref == 4:
                sv = r.s(); c = ("String", sv); ln = len(sv.encode("utf-16-le", "surrogatepass")) // 2
            elif ref == 5: c = ("Embed", r.s()); ln = 1
            elif ref == 6: c = ("Format", r.s(), r.s()); ln = 1
            elif ref == 7:
                tr = r.vu(); c = ("Type", tr, r.s() if tr in (3, 5) else None); ln = 1
            elif ref == 8: c = ("Any", [r.any() for _ in range(r.vu())]); ln = len(c[1])
            elif ref == 9: c = ("Doc", r.s(), r.any()); ln = 1
            else: raise ValueError(f"content ref {ref}")
            out.append(f"  {client}:{clock} len {ln} o={o} ro={ro} par={par} sub={sub} {c}")
            clock += ln
    ds = []
    for _ in range(r.vu()):
        client = r.vu()
        ds.append((client, [(r.vu(), r.vu()) for _ in range(r.vu())]))
    out.append(f"ds {ds}")
    return out


if __name__ == "__main__":
    a = sys.argv[1]
    try:
        data = open(a, "rb").read()
    except OSError:
        data = base64.b64decode(a)
    print("\n".join(dump_v1(data)))
