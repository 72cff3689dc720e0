#!/usr/bin/env python3
"""Regenerate the BN254 pairing constants hard-coded in csrc/pairing.hip from q, r, u
alone (no oracle import): twist Frobenius GAMMA_X/Y, the q^2-Frobenius constants of
Fq12 = Fq6[w]/(w^2-v), the hard-part exponent (q^4-q^2+1)/r and 6u+2."""
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
U = 4965661367192848881


def mul2(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def pow2(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = mul2(r, a)
        a = mul2(a, a)
        e >>= 1
    return r


def limbs(x, n=4):
    return ", ".join("0x%016xull" % ((x >> (64 * i)) & ((1 << 64) - 1)) for i in range(n))


def constants():
    xi = (9, 1)
    out = {"GAMMA_X": pow2(xi, (Q - 1) // 3), "GAMMA_Y": pow2(xi, (Q - 1) // 2)}
    out["FROB2"] = [pow2(xi, k * (Q * Q - 1) // 6) for k in range(6)]
    out["HARD"] = (Q ** 4 - Q ** 2 + 1) // R
    out["ATE"] = 6 * U + 2
    return out


if __name__ == "__main__":
    c = constants()
    for name in ("GAMMA_X", "GAMMA_Y"):
        print(name, "{", "{" + limbs(c[name][0]) + "},", "{" + limbs(c[name][1]) + "}", "}")
    for k, g in enumerate(c["FROB2"]):
        assert g[1] == 0
        print(f"FROB2[{k}]", "{" + limbs(g[0]) + "}")
    print("HARD", c["HARD"].bit_length(), "bits {" + limbs(c["HARD"], 12) + "}")
    print("ATE = 2^64 +", hex(c["ATE"] - (1 << 64)))
