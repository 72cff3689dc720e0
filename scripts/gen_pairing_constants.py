#!/usr/bin/env python3
"""Regenerate the BN254 pairing constants hard-coded in csrc/pairing.hip from q, r, u
alone (no oracle import): the q-Frobenius constants FROB1[k] = xi^(k(q-1)/6) (FROB1[2],
FROB1[3] are the twist Frobenius GAMMA_X/Y), the q^2-Frobenius constants of
Fq12 = Fq2[w]/(w^6-xi), R^3 mod q (R = 2^256), 6u+2 and u; also the hard-part exponent
(q^4-q^2+1)/r and its BN decomposition in powers of q with coefficients polynomial in u."""
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
    out["FROB1"] = [pow2(xi, k * (Q - 1) // 6) for k in range(6)]
    out["FROB2"] = [pow2(xi, k * (Q * Q - 1) // 6) for k in range(6)]
    out["R3"] = pow(2, 768, Q)
    out["HARD"] = (Q ** 4 - Q ** 2 + 1) // R
    out["HARD_LAMBDA"] = (-36 * U ** 3 - 30 * U ** 2 - 18 * U - 2, -36 * U ** 3 - 18 * U ** 2 - 12 * U + 1,
                          6 * U ** 2 + 1, 1)
    out["ATE"] = 6 * U + 2
    out["U"] = U
    return out


if __name__ == "__main__":
    c = constants()
    for k, g in enumerate(c["FROB1"]):
        print(f"FROB1[{k}]", "{", "{" + limbs(g[0]) + "},", "{" + limbs(g[1]) + "}", "}")
    for k, g in enumerate(c["FROB2"]):
        assert g[1] == 0
        print(f"FROB2[{k}]", "{" + limbs(g[0]) + "}")
    print("R3 {" + limbs(c["R3"]) + "}")
    print("U", hex(c["U"]))
    print("ATE = 2^64 +", hex(c["ATE"] - (1 << 64)))
