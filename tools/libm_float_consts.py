"""Where fate-llm_amd/csrc/fks_libm.h's fp32 libm-flavour constants come from: glibc's
__logf_data (e_logf_data.c: 16 {invc, logc} pairs, ln2, the 3-term polynomial) and
__sincosf_table[0] (sincosf_data.c: sign[4], 2/pi * 2^24, pi/2, then c0, c1, s1, c2, s2, c3,
s3, c4), read from the data of this image's libm.so.6 (glibc 2.35) by their shape.  Prints
them one float.hex() per line in the order `tests/libm_check consts` prints the header's;
tests/test_libm_float.py compares the two.  Test/provenance tooling: nothing shipped reads it.

  python tools/libm_float_consts.py [/lib/x86_64-linux-gnu/libm.so.6]"""
import struct
import sys

LN2 = float.fromhex("0x1.62e42fefa39efp-1")
HPI = float.fromhex("0x1.921fb54442d18p+0")


def _d(b, off, n):
    return list(struct.unpack_from(f"<{n}d", b, off))


def find_logf(b):
    key = struct.pack("<d", LN2)
    i = b.find(key)
    while i >= 0:
        tab = _d(b, i - 256, 32)
        poly = _d(b, i + 8, 3)
        if all(0.6 < tab[2 * j] < 1.5 for j in range(16)) and -0.3 < poly[0] < -0.2 and -0.6 < poly[2] < -0.4:
            return tab, LN2, poly
        i = b.find(key, i + 1)
    raise LookupError("__logf_data not found")


def find_sincosf(b):
    key = struct.pack("<d", HPI)
    i = b.find(key)
    while i >= 0:
        head = _d(b, i - 40, 5)
        if head[:4] == [1.0, -1.0, -1.0, 1.0] and abs(head[4] - 2 / 3.141592653589793 * 2**24) < 1:
            return head[4], HPI, _d(b, i + 8, 8)  # c0, c1, s1, c2, s2, c3, s3, c4
        i = b.find(key, i + 1)
    raise LookupError("__sincosf_table not found")


def constants(path="/lib/x86_64-linux-gnu/libm.so.6"):
    b = open(path, "rb").read()
    tab, ln2, poly = find_logf(b)
    hpi_inv, hpi, sc = find_sincosf(b)
    return tab + [ln2] + poly + [hpi_inv, hpi] + sc


if __name__ == "__main__":
    for v in constants(*sys.argv[1:]):
        print(float(v).hex())
