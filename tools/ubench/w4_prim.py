"""Check tools/ubench/w4_prim's output file with Python integers (engine form: x 2^384)."""
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RI = pow(1 << 384, -1, P)
NOUT, n, NIN = 84, 16, 12
raw = open(sys.argv[1] if len(sys.argv) > 1 else "w4_prim.bin", "rb").read()
vals = [int.from_bytes(raw[48 * i:48 * i + 48], "little") for i in range(len(raw) // 48)]
ins, outs = vals[:NIN * n], vals[NIN * n:]
names = ["a0b0", "a1b1", "kara0", "kara1", "sqr0", "sqr1"] + ["sub%d" % k for k in range(1, 11)] + [
    "3a0", "8a1", "a0/2", "a0+b1", "3a0*(a1-b1)", "8a0*8b0", "bias1", "bias10"] + ["dbl%d" % i for i in range(6)] + ["add%d" % i for i in range(6)] + [
    "%s.%d" % (nm, k) for nm in ["A", "B", "E", "C", "F", "XB2", "D", "X3", "u", "Eu", "YZ", "C8"] for k in range(2)] + [
    "copy%d" % i for i in range(6)] + ["dblB%d" % i for i in range(6)] + ["dblT%d" % i for i in range(6)] + ["T.A1", "T.C1", "T.F1", "T.XB2_1", "T.D1", "T.X3_1"]
def f2(a, b):
    return (a % P, b % P)


def mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def lin(*terms):
    return tuple(sum(k * t[i] for k, t in terms) % P for i in range(2))


def dbl(X, Y, Z):
    A, B = mul(X, X), mul(Y, Y)
    C = mul(B, B)
    XB = lin((1, X), (1, B))
    D = lin((2, mul(XB, XB)), (-2, A), (-2, C))
    E = lin((3, A))
    F = mul(E, E)
    X3 = lin((1, F), (-2, D))
    Y3 = lin((1, mul(E, lin((1, D), (-1, X3)))), (-8, C))
    Z3 = lin((2, mul(Y, Z)))
    return X3, Y3, Z3


def add(X1, Y1, Z1, X2, Y2, Z2):
    Z1Z1, Z2Z2 = mul(Z1, Z1), mul(Z2, Z2)
    U1, U2 = mul(X1, Z2Z2), mul(X2, Z1Z1)
    S1, S2 = mul(mul(Y1, Z2), Z2Z2), mul(mul(Y2, Z1), Z1Z1)
    H = lin((1, U2), (-1, U1))
    I = mul(lin((2, H)), lin((2, H)))
    J = mul(H, I)
    r = lin((2, S2), (-2, S1))
    V = mul(U1, I)
    X3 = lin((1, mul(r, r)), (-1, J), (-2, V))
    Y3 = lin((1, mul(r, lin((1, V), (-1, X3)))), (-2, mul(S1, J)))
    zz = lin((1, mul(lin((1, Z1), (1, Z2)), lin((1, Z1), (1, Z2)))), (-1, Z1Z1), (-1, Z2Z2))
    Z3 = mul(zz, H)
    return X3, Y3, Z3


bad = {}
for w in range(n):
    x = [ins[NIN * w + i] * RI % P for i in range(NIN)]
    a0, a1, b0, b1 = x[:4]
    want = [a0 * b0, a1 * b1, a0 * b0 - a1 * b1, a0 * b1 + a1 * b0, a0 * a0 - a1 * a1, 2 * a0 * a1]
    want += [a0 - b0] * 10
    want += [3 * a0, 8 * a1, a0 * pow(2, -1, P), a0 + b1, 3 * a0 * (a1 - b1), 64 * a0 * b0, 2 * P, 1024 * P]
    want += [c for q in dbl(f2(x[0], x[1]), f2(x[2], x[3]), f2(x[4], x[5])) for c in q]
    want += [c for q in add(f2(x[0], x[1]), f2(x[2], x[3]), f2(x[4], x[5]), f2(x[6], x[7]), f2(x[8], x[9]), f2(x[10], x[11])) for c in q]
    X, Y, Z = f2(x[0], x[1]), f2(x[2], x[3]), f2(x[4], x[5])
    A, B = mul(X, X), mul(Y, Y)
    E = lin((3, A))
    C, F = mul(B, B), mul(E, E)
    XB = lin((1, X), (1, B))
    XB2 = mul(XB, XB)
    D = lin((2, XB2), (-2, A), (-2, C))
    X3 = lin((1, F), (-2, D))
    u = lin((1, D), (-1, X3))
    Eu = mul(E, u)
    YZ = mul(Y, Z)
    C8 = lin((8, C))
    for q in (A, B, E, C, F, XB2, D, X3, u, Eu, YZ, C8):
        want += list(q)
    want += [c for q in dbl(X, Y, Z) for c in q] * 3
    want += [A[1], C[1], F[1], XB2[1], D[1], X3[1]]
    for i in range(NOUT):
        got = outs[NOUT * w + i]
        exp = want[i] % P * (1 << 384) % P
        if got != exp:
            bad.setdefault(names[i], 0)
            bad[names[i]] += 1
print("mismatches by op:", bad if bad else "none")
