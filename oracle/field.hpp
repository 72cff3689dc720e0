// ORACLE — TEST INFRASTRUCTURE ONLY.
// CPU restatement of adria0/plonk-by-fingers (reference @ /root/reference, Rust).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this code, and only as the checker. The product path (libpbf.so) never links it.
//
// Restates src/utils/u64field.rs: U64Field<M>, canonical residues in [0, M).
#pragma once
#include <cstdint>
#include <string>

namespace oracle {

typedef unsigned __int128 u128;
typedef __int128 i128;

// u64field.rs:10-25 extended_gcd (i64 there). Widened to i128 so the restatement
// also covers moduli >= 2^63 (Goldilocks), where the reference's `M as i64` cannot
// represent M; for M < 2^63 the result is identical (the inverse is unique).
inline void extended_gcd(i128 a, i128 b, i128& g, i128& s_out) {
  i128 s = 0, old_s = 1, r = b, old_r = a;
  while (r != 0) {
    i128 q = old_r / r;
    i128 t = old_r - q * r; old_r = r; r = t;
    t = old_s - q * s; old_s = s; s = t;
  }
  g = old_r; s_out = old_s;
}

// A U64Field element whose modulus is a type parameter: Mod::m() -> uint64_t.
// Arithmetic is the mathematically defined result of the reference's formulas
// (u64field.rs:107-228). The reference computes (a*b)%M in u64, which is exact
// only for M < 2^32 (u64field.rs:177); here the product is taken in u128 so the
// same formulas stay exact for 64-bit moduli.
template <class Mod>
struct Fe {
  uint64_t v;
  Fe() : v(0) {}
  static Fe raw(uint64_t x) { Fe f; f.v = x; return f; }
  // u64field.rs:95-99  From<u64>: n % M
  static Fe from_u64(uint64_t n) { return raw(n % Mod::m()); }
  // u64field.rs:85-93  From<i64>: negative -> -(|n|)
  static Fe from_i64(int64_t n) {
    if (n < 0) return -from_u64((uint64_t)(-(i128)n));
    return from_u64((uint64_t)n);
  }
  static Fe zero() { return raw(0); }
  static Fe one() { return from_u64(1); }
  static uint64_t order() { return Mod::m(); }
  bool is_zero() const { return v == 0; }
  uint64_t as_u64() const { return v; }
  bool in_field() const { return v < Mod::m(); }  // u64field.rs:49-51
  // u64field.rs:107-112 add: (a+b) % M (u128 to stay exact for M >= 2^63)
  Fe operator+(Fe o) const { return raw((uint64_t)(((u128)v + o.v) % Mod::m())); }
  // u64field.rs:160-165 neg: (M - a) % M
  Fe operator-() const { return raw((Mod::m() - v) % Mod::m()); }
  // u64field.rs:147-152 sub = a + (-b)
  Fe operator-(Fe o) const { return *this + (-o); }
  // u64field.rs:174-179 mul: (a*b) % M
  Fe operator*(Fe o) const { return raw((uint64_t)(((u128)v * o.v) % Mod::m())); }
  Fe& operator+=(Fe o) { *this = *this + o; return *this; }
  Fe& operator-=(Fe o) { *this = *this - o; return *this; }
  Fe& operator*=(Fe o) { *this = *this * o; return *this; }
  bool operator==(Fe o) const { return v == o.v; }
  bool operator!=(Fe o) const { return v != o.v; }
  bool operator<(Fe o) const { return v < o.v; }
  // u64field.rs:52-63 inv via extended gcd; `ok=false` mirrors the `None` branch.
  Fe inv(bool& ok) const {
    i128 g, c;
    extended_gcd((i128)v, (i128)Mod::m(), g, c);
    if (g != 1) { ok = false; return zero(); }
    ok = true;
    if (c < 0) return raw((uint64_t)((i128)Mod::m() + c));
    return raw((uint64_t)c);
  }
  Fe inv_unwrap() const {
    bool ok; Fe r = inv(ok);
    if (!ok) throw std::string("inv of non-invertible element (reference panics on unwrap)");
    return r;
  }
  // u64field.rs:222-228 div: rhs.inv().map(|v| v*self)
  Fe div(Fe rhs, bool& ok) const { Fe i = rhs.inv(ok); return ok ? i * *this : zero(); }
  Fe div_unwrap(Fe rhs) const { return rhs.inv_unwrap() * *this; }
  // u64field.rs:64-75 pow: LSB-first square-and-multiply
  Fe pow(uint64_t e) const {
    Fe r = one(), b = *this;
    while (e > 0) {
      if (e & 1) r = r * b;
      e >>= 1;
      b = b * b;
    }
    return r;
  }
};

template <uint64_t M>
struct StaticMod { static uint64_t m() { return M; } };

// Runtime modulus (used behind the C API where M is an argument).
struct DynMod {
  static uint64_t& ref() { static thread_local uint64_t M = 0; return M; }
  static uint64_t m() { return ref(); }
};

typedef Fe<DynMod> DF;
static const uint64_t GOLDILOCKS_P = 0xFFFFFFFF00000001ull;

}  // namespace oracle
