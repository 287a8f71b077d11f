"""Check r28_bench's `check` output: each line is a, b, r as 14 hex limbs of 28 bits;
r must equal a*b*2^-392 mod p up to one multiple of p, and be < 2p."""
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RINV = pow(2, -392, P)


def val(s):
    return sum(int(x, 16) << (28 * i) for i, x in enumerate(s.split(",")))


bad = n = 0
for line in open(sys.argv[1]):
    a, b, r = (val(x) for x in line.split())
    n += 1
    if r % P != a * b * RINV % P or r >= 2 * P:
        bad += 1
print("r28 check: %d products, %d wrong" % (n, bad))
sys.exit(1 if bad or not n else 0)
