"""Check r28_bench's `check` / `check2` output: each line is a, b, r (or a0 a1 b0 b1 r0 r1)
as 14 hex limbs of 28 bits; r must equal the product times 2^-392 mod p and be < 2p."""
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RINV = pow(2, -392, P)


def val(s):
    return sum(int(x, 16) << (28 * i) for i, x in enumerate(s.split(",")))


bad = n = 0
for line in open(sys.argv[1]):
    v = [val(x) for x in line.split()]
    n += 1
    if len(v) == 3:  # Fp product
        a, b, r = v
        ok = r % P == a * b * RINV % P and r < 2 * P
    else:  # Fp2 product (u^2 = -1)
        a0, a1, b0, b1, r0, r1 = v
        ok = (r0 % P == (a0 * b0 - a1 * b1) * RINV % P and r1 % P == (a0 * b1 + a1 * b0) * RINV % P
              and r0 < 2 * P and r1 < 2 * P)
    bad += not ok
print("r28 check: %d products, %d wrong" % (n, bad))
sys.exit(1 if bad or not n else 0)
