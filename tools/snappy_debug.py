"""Debug helper: decode generated snappy streams on the GPU and report, for the
first wrong byte, the tag that produced it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import test_snappy as T  # noqa: E402


def tags_of(src):
    """(tag start, kind, output start, length, offset) of every tag."""
    i = 0
    while src[i] & 0x80:
        i += 1
    i += 1
    d, out = 0, []
    while i < len(src):
        t = src[i]
        if t & 3 == 0:
            x = t >> 2
            if x < 60:
                h, ln = 1, x + 1
            else:
                nb = x - 59
                h, ln = 1 + nb, int.from_bytes(src[i + 1:i + 1 + nb], "little") + 1
            out.append((i, "lit", d, ln, 0))
            i += h + ln
        elif t & 3 == 1:
            ln, off = 4 + ((t >> 2) & 7), (t & 0xE0) << 3 | src[i + 1]
            out.append((i, "c1", d, ln, off))
            i += 2
        elif t & 3 == 2:
            ln, off = 1 + (t >> 2), src[i + 1] | src[i + 2] << 8
            out.append((i, "c2", d, ln, off))
            i += 3
        else:
            ln, off = 1 + (t >> 2), int.from_bytes(src[i + 1:i + 5], "little")
            out.append((i, "c4", d, ln, off))
            i += 5
        d += ln
    return out


def main():
    import pqgpu
    dec = pqgpu.GpuDecoder(0)
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
    for name, kw in [("nofar", dict(far_frac=0.0)), ("far", dict(far_frac=0.6)), ("lit8", dict(lit_max=8)),
                     ("default", {})]:
        src, plain = T.stream(rng, 60_000, **kw)
        rc, got = T._gpu(dec, src)
        bad = next((i for i in range(min(len(got), len(plain))) if got[i] != plain[i]), None)
        print(name, "rc", rc, "len", len(got), len(plain), "first bad", bad)
        if bad is not None:
            tg = tags_of(src)
            for k, (pos, kind, d, ln, off) in enumerate(tg):
                if d <= bad < d + ln:
                    print("  tag", k, "at", pos, kind, "out", d, "len", ln, "off", off,
                          "src byte", bad - off if off else None)
                    for j in range(max(0, k - 3), min(len(tg), k + 3)):
                        print("   ", tg[j])
                    break
            nbad = sum(1 for i in range(min(len(got), len(plain))) if got[i] != plain[i])
            print("  wrong bytes:", nbad)
    dec.close()


if __name__ == "__main__":
    main()
