"""Check tools/microbench/f64mul's products (`f64mul verify`) against Python big integers:
out = x * y mod p as a value < 2^260 in five limbs < 2^52 (p = 2^256 - 2^32 - 977).
Usage: python tools/microbench/f64mul_check.py f64mul_verify.bin"""
import struct
import sys

P = 2**256 - 2**32 - 977


def main():
    raw = open(sys.argv[1], "rb").read()
    n = struct.unpack_from("<I", raw)[0]
    q = struct.unpack_from("<%dQ" % (15 * n), raw, 4)
    xs, ys, os_ = q[:5 * n], q[5 * n:10 * n], q[10 * n:]

    def val(a, i):
        return sum(a[5 * i + k] << (52 * k) for k in range(5))
    bad = 0
    for i in range(n):
        x, y, o = val(xs, i), val(ys, i), val(os_, i)
        limbs_ok = all(os_[5 * i + k] < (1 << 52) for k in range(5))
        if not limbs_ok or o >= (1 << 260) or o % P != (x * y) % P:
            bad += 1
            if bad < 5:
                print("mismatch lane", i, hex(x), hex(y), hex(o))
    print('{"products": %d, "mismatches": %d}' % (n, bad))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
