#!/usr/bin/env python3
"""Constants of the 29-bit-limb Montgomery arithmetic of csrc/msm_l29.hpp (BN254 Fq,
R = 2^261): p's limbs, -p^-1 mod 2^29, 8p and 16p in redundant limbs (every limb >= 2^31 - 4
below the top, so a + M - b never borrows for normalised b), and the domain constants
2^266, 2^271, 2^256, 2^251 mod p, and 12p, 4p in normalised limbs (round 6: the values added
at 2^261 by l29::mul_shift_sub). Prints the C++ block; tests/test_l29_constants.py checks
the header against this script."""
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617  # BN254 Fr
MASK = (1 << 29) - 1


def limbs(v, k=9):
    out = []
    for _ in range(k):
        out.append(v & MASK)
        v >>= 29
    assert v == 0
    return out


def redundant(mult):
    n = limbs(mult * P)
    m = [n[0] + (1 << 31)] + [n[i] + (1 << 31) - 4 for i in range(1, 8)] + [n[8] - 4]
    assert sum(x << (29 * i) for i, x in enumerate(m)) == mult * P
    assert all(0 <= x < (1 << 32) for x in m)
    return m


def redundant_r(mult, a):
    """mult r with 2^a added to limbs 0..7 and 2^(a-29) taken from the next limb: every limb but
    the top at least 2^a - 2^(a-29), so x + B - y never borrows for y's limbs below that"""
    n = limbs(mult * R)
    m = [n[0] + (1 << a)] + [n[i] + (1 << a) - (1 << (a - 29)) for i in range(1, 8)] + [n[8] - (1 << (a - 29))]
    assert sum(x << (29 * i) for i, x in enumerate(m)) == mult * R
    assert all(0 <= x < (1 << 32) for x in m)
    return m


def fr_constants():
    """csrc/fr29.hpp (round 6: the Fr NTT passes on 29-bit limbs, R' = 2^261)"""
    return {
        "R29": limbs(R),
        "NR29": [(-pow(R, -1, 1 << 29)) % (1 << 29)],
        "QC": [(1 << 264) // R],
        "B4R": redundant_r(4, 29),
        "B8R": redundant_r(8, 30),
        "B2R": redundant_r(2, 29),
    }


def constants():
    return {
        "P29": limbs(P),
        "NP29": [(-pow(P, -1, 1 << 29)) % (1 << 29)],
        "M8P": redundant(8),
        "M16P": redundant(16),
        "C266": limbs(pow(2, 266, P)),
        "C271": limbs(pow(2, 271, P)),
        "C256": limbs(pow(2, 256, P)),
        "C251": limbs(pow(2, 251, P)),
        "P12": limbs(12 * P),
        "P4": limbs(4 * P),
    }


def main():
    for name, v in list(constants().items()) + list(fr_constants().items()):
        vals = ", ".join(f"0x{x:08x}u" for x in v)
        if len(v) == 1:
            print(f"constexpr uint32_t {name} = {vals};")
        else:
            print(f"constexpr uint32_t {name}[9] = {{{vals}}};")


if __name__ == "__main__":
    main()
