// ge25519.h -- edwards25519 group arithmetic for gfx950 (one point per lane).
//
// Coordinates follow the extended/"p1p1" scheme of the twisted-Edwards
// formulas (Hisil-Wong-Carter-Dawson 2008, a = -1):
//   p2     (X:Y:Z)           x = X/Z, y = Y/Z               -- doubling input
//   p3     (X:Y:Z:T)         + T = XY/Z                     -- addition input
//   p1p1   (X:Y:Z:T)         x = X/Z, y = Y/T               -- op output
//   cached (Y+X, Y-X, Z, 2dT)                               -- per-lane tables
//   niels  (y+x, y-x, 2dxy), Z = 1                          -- fixed B table
// Only canonical encodings of results are ever compared, so equality with
// libsodium's ref10 is a property of the group, not
// of the formulas.  Decoding and the acceptance predicates below restate
// libsodium 1.0.18 exactly.
#pragma once
#include "fe25519.h"
#include "modinv.h"

namespace ouro {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YplusX, YminusX, Z2, T2d; };  // Z2 = 2Z
struct ge_niels { fe yplusx, yminusx, xy2d; };

// Limb-bound profile the formulas keep (unit = one reduced element, see
// fe25519.h; the host bound tracker checks every case):
//   p2 / p3 inputs: X <= 2, Y, Z, T <= 1 (X may be a negation)
//   p1p1 outputs:   X <= 3, Y <= 2, Z <= 3, T <= 4
//   cached:         Y+X <= 3, Y-X <= 3, Z2 <= 2, 2dT <= 1
// and every product puts the narrower operand second (fe_mul's 19 g < 2^32).

OURO_FI ge_p3 ge_p3_identity() { return ge_p3{fe_zero(), fe_one(), fe_one(), fe_zero()}; }
OURO_FI ge_p2 ge_p2_identity() { return ge_p2{fe_zero(), fe_one(), fe_one()}; }
OURO_FI ge_cached ge_cached_identity() {
  return ge_cached{fe_one(), fe_one(), fe_two(), fe_zero()};
}
OURO_FI ge_niels ge_niels_identity() { return ge_niels{fe_one(), fe_one(), fe_zero()}; }

OURO_FI ge_p2 ge_p1p1_to_p2(const ge_p1p1& p) {
  ge_p2 r;
  fe_mul_x2(r.X, r.Y, p.T, p.X, p.Z, p.Y);
  r.Z = fe_mul(p.T, p.Z);
  return r;
}
OURO_FI ge_p3 ge_p1p1_to_p3(const ge_p1p1& p) {
  ge_p3 r;
  fe_mul_x2(r.X, r.Y, p.T, p.X, p.Z, p.Y);
  fe_mul_x2(r.Z, r.T, p.T, p.Z, p.X, p.Y);
  return r;
}
OURO_FI ge_p2 ge_p3_to_p2(const ge_p3& p) { return ge_p2{p.X, p.Y, p.Z}; }
OURO_FI ge_cached ge_p3_to_cached(const ge_p3& p) {
  return ge_cached{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), fe_add(p.Z, p.Z), fe_mul(p.T, fe_d2())};
}

// 2P: A = X^2, B = Y^2, C = 2Z^2; x' = 2XY / (B - A), y' = (A + B) / (C - (B - A)).
// A + B is re-normalised (fe_carry) so that X' = (X+Y)^2 - (A+B) stays within 3.
OURO_FI ge_p1p1 ge_p2_dbl(const ge_p2& p) {
  fe A = fe_sq(p.X);
  fe B = fe_sq(p.Y);
  fe C = fe_sq2(p.Z);
  fe S = fe_sq(fe_add(p.X, p.Y));
  ge_p1p1 r;
  r.Y = fe_carry(fe_add(B, A));
  r.Z = fe_sub(B, A);
  r.X = fe_sub(S, r.Y);
  r.T = fe_sub(fe_add(C, A), B);
  return r;
}
OURO_FI ge_p1p1 ge_p3_dbl(const ge_p3& p) { return ge_p2_dbl(ge_p3_to_p2(p)); }

// ge_p2_dbl(ge_p1p1_to_p2(t)) -- a doubling of a chain -- with the three
// products of the p2 conversion in lockstep, then the four squarings in
// lockstep (fe25519.h fe_mul_xn / fe_sq_xn): the same operations and operand
// order, so the same bounds, scheduled so no multiply-add waits on the one
// before it (round 4: 29.3 -> 25.9 ps per chip-wide doubling at two waves per
// SIMD, profiles/r04/occupancy_lockstep.json).
// OURO_DBL_COMP (device, the default since round 6): the doubling returns
// (X, Z) negated -- X = Y' - S, Z = A - B, the same point -- so that S, used
// only there, comes out of its squaring complemented (fe_sq_xn kComp) and
// X = Y' + (mask - S) + (2p - mask) is one three-input add per limb: the
// limbs are exactly fe_sub(Y', S)'s, ~10 VALU fewer per doubling.  The host
// build (and OURO_DBL_COMP=0) computes the same limbs with fe_sub.
#ifndef OURO_DBL_COMP
#define OURO_DBL_COMP 1
#endif
OURO_FI ge_p1p1 ge_dbl_lockstep(const ge_p1p1& t) {
  const fe f[3] = {t.T, t.Z, t.T}, g[3] = {t.X, t.Y, t.Z};
  fe p[3];
  fe_mul_xn<3>(p, f, g);  // X = T X, Y = Z Y, Z = T Z
  const fe in[4] = {p[0], p[1], p[2], fe_add(p[0], p[1])};
  constexpr int kScale[4] = {1, 1, 2, 1};  // A = X^2, B = Y^2, C = 2 Z^2, S = (X + Y)^2
  fe o[4];
  ge_p1p1 r;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (OURO_DBL_COMP) {
    fe_sq_xn<4, 8u>(o, in, kScale);  // o[3] = mask - S
    r.Y = fe_carry(fe_add(o[1], o[0]));
    r.Z = fe_sub(o[0], o[1]);
#pragma unroll
    for (int i = 0; i < 10; i++)
      r.X.v[i] = r.Y.v[i] + o[3].v[i] + (kp_limb(2, i) - limb_mask(i));
    r.T = fe_sub(fe_add(o[2], o[0]), o[1]);
    return r;
  }
#endif
  fe_sq_xn<4>(o, in, kScale);
  r.Y = fe_carry(fe_add(o[1], o[0]));
  r.Z = OURO_DBL_COMP ? fe_sub(o[0], o[1]) : fe_sub(o[1], o[0]);
  r.X = OURO_DBL_COMP ? fe_sub(r.Y, o[3]) : fe_sub(o[3], r.Y);
  r.T = fe_sub(fe_add(o[2], o[0]), o[1]);
  return r;
}

// P + Q (neg = false) or P - Q (neg = true), Q cached.  The sign is a per-lane
// select so a wave stays convergent whatever the digits are.  affine_q (wave-
// uniform): Q has Z = 1 (Z2 = 2), so 2 Z_P Z_Q is a re-normalised addition.
OURO_FI ge_p1p1 ge_add_cached(const ge_p3& p, const ge_cached& q, bool neg,
                              bool affine_q = false) {
  fe qa = fe_select(q.YminusX, q.YplusX, neg);
  fe qb = fe_select(q.YplusX, q.YminusX, neg);
  fe A, B, C, D;
  fe_mul_x2(A, B, fe_add(p.Y, p.X), qa, fe_sub(p.Y, p.X), qb);
  if (affine_q) {
    C = fe_mul(p.T, q.T2d);
    D = fe_carry(fe_add(p.Z, p.Z));
  } else {
    fe_mul_x2(C, D, p.T, q.T2d, p.Z, q.Z2);
  }
  fe Dp = fe_add(D, C), Dm = fe_sub(D, C);
  ge_p1p1 r;
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_select(Dm, Dp, neg);
  r.T = fe_select(Dp, Dm, neg);
  return r;
}

// ge_add_cached(ge_p1p1_to_p3(t), q, neg, affine_q) -- a chain's addition --
// with the four products of the p3 conversion in lockstep, then the
// addition's four (three for an affine q) in lockstep (fe_mul_xn), the same
// operands in the same order as the two calls (the same bounds), like the
// doubling's ge_dbl_lockstep (A/B switch OURO_ADD_LOCKSTEP, verify.h)
// kPair: the products two at a time (fewer live registers) instead of all at once
template <bool kPair = false>
OURO_FI ge_p1p1 ge_add_lockstep(const ge_p1p1& t, const ge_cached& q, bool neg, bool affine_q) {
  const fe f1[4] = {t.T, t.Z, t.T, t.X}, g1[4] = {t.X, t.Y, t.Z, t.Y};
  fe p[4];
  if (kPair) {  // X = T X, Y = Z Y, Z = T Z, T = X Y
    fe_mul_xn<2>(p, f1, g1);
    fe_mul_xn<2>(p + 2, f1 + 2, g1 + 2);
  } else {
    fe_mul_xn<4>(p, f1, g1);
  }
  const fe qa = fe_select(q.YminusX, q.YplusX, neg);
  const fe qb = fe_select(q.YplusX, q.YminusX, neg);
  fe o[4];
  const fe f2[4] = {fe_add(p[1], p[0]), fe_sub(p[1], p[0]), p[3], p[2]};
  const fe g2[4] = {qa, qb, q.T2d, q.Z2};
  if (affine_q) {
    if (kPair) {
      fe_mul_xn<2>(o, f2, g2);
      o[2] = fe_mul(f2[2], g2[2]);
    } else {
      fe_mul_xn<3>(o, f2, g2);
    }
    o[3] = fe_carry(fe_add(p[2], p[2]));
  } else if (kPair) {
    fe_mul_xn<2>(o, f2, g2);
    fe_mul_xn<2>(o + 2, f2 + 2, g2 + 2);
  } else {
    fe_mul_xn<4>(o, f2, g2);
  }
  const fe Dp = fe_add(o[3], o[2]), Dm = fe_sub(o[3], o[2]);
  ge_p1p1 r;
  r.X = fe_sub(o[0], o[1]);
  r.Y = fe_add(o[0], o[1]);
  r.Z = fe_select(Dm, Dp, neg);
  r.T = fe_select(Dp, Dm, neg);
  return r;
}

// ---- lane-quad group operations (latency mode) --------------------------------
// Four consecutive lanes (one DPP quad) hold the same point and split the
// independent field products of one group operation: lane q = threadIdx.x & 3
// computes product q, then every lane reads all four through quad_perm
// broadcasts.  A doubling or an addition then costs one product's time
// instead of three or four on the critical lane of a small window.
// Bounds: a lane's operand is one of four candidates, so the worst case of
// each operand is the largest of its candidates' -- the host build (which
// runs the four products in sequence) gives every emulated product exactly
// those merged bounds, so test_zero_bound_violations covers these formulas.
struct fe4 { fe v[4]; };

#if defined(__HIP_DEVICE_COMPILE__)
// per-limb v_cndmask with a constant lane mask (lanes in `mask` take b).  In
// asm so LLVM cannot turn a select of four elements into a scratch array
// indexed by the lane.
constexpr uint64_t kQuadOdd = 0xaaaaaaaaaaaaaaaaull;   // quad position 1, 3
constexpr uint64_t kQuadHigh = 0xccccccccccccccccull;  // quad position 2, 3
OURO_FI fe fe_sel_lanes(const fe& a, const fe& b, uint64_t mask) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++)
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(h.v[i]) : "v"(a.v[i]), "v"(b.v[i]), "s"(mask));
  return h;
}
OURO_FI fe fe_quad_pick(const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
  return fe_sel_lanes(fe_sel_lanes(a0, a1, kQuadOdd), fe_sel_lanes(a2, a3, kQuadOdd), kQuadHigh);
}
template <int J>
OURO_FI fe fe_quad_bcast(const fe& f) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++)
    h.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)f.v[i], J * 0x55, 0xf, 0xf, true);
  return h;
}
OURO_FI fe4 fe_quad_gather(const fe& m) {
  return fe4{{fe_quad_bcast<0>(m), fe_quad_bcast<1>(m), fe_quad_bcast<2>(m), fe_quad_bcast<3>(m)}};
}
#else
// candidate j with the bounds of the largest candidate (see above)
OURO_FI fe fe_quad_merged(const fe4& a, int j) {
  fe r = a.v[j];
  OURO_TRK(for (int i = 0; i < 10; i++) for (int k = 0; k < 4; k++) if (a.v[k].b[i] > r.b[i])
               r.b[i] = a.v[k].b[i];)
  return r;
}
#endif

// out.v[j] = a.v[j] * b.v[j]
OURO_FI fe4 fe_mul_quad(const fe4& a, const fe4& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fe_quad_gather(fe_mul(fe_quad_pick(a.v[0], a.v[1], a.v[2], a.v[3]),
                               fe_quad_pick(b.v[0], b.v[1], b.v[2], b.v[3])));
#else
  fe4 r;
  for (int j = 0; j < 4; j++) r.v[j] = fe_mul(fe_quad_merged(a, j), fe_quad_merged(b, j));
  return r;
#endif
}
#if defined(__HIP_DEVICE_COMPILE__)
// this lane's x^2 (2 x^2 on quad position 2), gathered
OURO_FI fe4 fe_sq_quad_dbl2_own(const fe& x) {
  uint64_t t[10];
  fe_sq_cols(t, x);
  const uint32_t sh = (threadIdx.x & 3u) == 2u ? 1u : 0u;
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] <<= sh;
  return fe_quad_gather(fe_carry64(t));
}
#endif
// out.v[j] = a.v[j]^2, except out.v[2] = 2 a.v[2]^2
OURO_FI fe4 fe_sq_quad_dbl2(const fe4& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fe_sq_quad_dbl2_own(fe_quad_pick(a.v[0], a.v[1], a.v[2], a.v[3]));
#else
  fe4 r;
  for (int j = 0; j < 4; j++) {
    const fe x = fe_quad_merged(a, j);
    r.v[j] = j == 2 ? fe_sq2(x) : fe_sq(x);
  }
  return r;
#endif
}
// the products of the p1p1 conversions: (T X, Z Y, T Z, X Y)
OURO_FI fe4 ge_p1p1_products_quad(const ge_p1p1& p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const fe a = fe_sel_lanes(p.T, fe_sel_lanes(p.Z, p.X, kQuadHigh), kQuadOdd);
  const fe b = fe_sel_lanes(fe_sel_lanes(p.X, p.Z, kQuadHigh), p.Y, kQuadOdd);
  return fe_quad_gather(fe_mul(a, b));
#else
  return fe_mul_quad(fe4{{p.T, p.Z, p.T, p.X}}, fe4{{p.X, p.Y, p.Z, p.Y}});
#endif
}

OURO_FI ge_p2 ge_p1p1_to_p2_quad(const ge_p1p1& p) {
  const fe4 m = ge_p1p1_products_quad(p);
  return ge_p2{m.v[0], m.v[1], m.v[2]};
}
OURO_FI ge_p3 ge_p1p1_to_p3_quad(const ge_p1p1& p) {
  const fe4 m = ge_p1p1_products_quad(p);
  return ge_p3{m.v[0], m.v[1], m.v[2], m.v[3]};
}
// the doubling formula from the four squares A = X^2, B = Y^2, C = 2 Z^2,
// S = (X + Y)^2 (every lane holds all four)
OURO_FI ge_p1p1 ge_dbl_from_squares(const fe4& s) {
  const fe &A = s.v[0], &B = s.v[1], &C = s.v[2], &S = s.v[3];
  ge_p1p1 r;
  r.Y = fe_carry(fe_add(B, A));
  r.Z = fe_sub(B, A);
  r.X = fe_sub(S, r.Y);
  r.T = fe_sub(fe_add(C, A), B);
  return r;
}
// ge_p2_dbl with its four squarings on the four lanes
OURO_FI ge_p1p1 ge_p2_dbl_quad(const ge_p2& p) {
  return ge_dbl_from_squares(fe_sq_quad_dbl2(fe4{{p.X, p.Y, p.Z, fe_add(p.X, p.Y)}}));
}
// 2 * (p1p1 point): the p2 conversion's products X, Y, Z stay on quad
// positions 0, 1, 2, which are exactly the squaring inputs those positions
// need; position 3 adds X + Y from its neighbours -- no gather, no pick
OURO_FI ge_p1p1 ge_dbl_from_p1p1_quad(const ge_p1p1& t) {
#if defined(__HIP_DEVICE_COMPILE__)
  const fe a = fe_sel_lanes(t.T, fe_sel_lanes(t.Z, t.X, kQuadHigh), kQuadOdd);
  const fe b = fe_sel_lanes(fe_sel_lanes(t.X, t.Z, kQuadHigh), t.Y, kQuadOdd);
  const fe m = fe_mul(a, b);  // position 0: X, 1: Y, 2: Z, 3: (unused) X Y
  const uint32_t pos3 = (threadIdx.x & 3u) == 3u ? 0xffffffffu : 0u;
  fe in;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    // quad_perm [0,1,2,0]: own product, position 3 takes X; [1,1,1,1]: Y
    const uint32_t own = (uint32_t)__builtin_amdgcn_mov_dpp((int)m.v[i], 0x24, 0xf, 0xf, true);
    const uint32_t y = (uint32_t)__builtin_amdgcn_mov_dpp((int)m.v[i], 0x55, 0xf, 0xf, true);
    in.v[i] = own + (y & pos3);
  }
  return ge_dbl_from_squares(fe_sq_quad_dbl2_own(in));
#else
  return ge_p2_dbl_quad(ge_p1p1_to_p2_quad(t));
#endif
}
// ge_add_cached with its four products on the four lanes; an affine Q carries
// Z2 = 2, so D = 2 Z_P either way
OURO_FI ge_p1p1 ge_add_cached_quad(const ge_p3& p, const ge_cached& q, bool neg) {
  const fe qa = fe_select(q.YminusX, q.YplusX, neg);
  const fe qb = fe_select(q.YplusX, q.YminusX, neg);
  const fe4 m = fe_mul_quad(fe4{{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), p.T, p.Z}},
                            fe4{{qa, qb, q.T2d, q.Z2}});
  const fe &A = m.v[0], &B = m.v[1], &C = m.v[2], &D = m.v[3];
  const fe Dp = fe_add(D, C), Dm = fe_sub(D, C);
  ge_p1p1 r;
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_select(Dm, Dp, neg);
  r.T = fe_select(Dp, Dm, neg);
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// P + Q for a p1p1 P, each lane holding only its own operand of Q (quad
// position 0: Y+X or Y-X of Q as the sign asks, 1: the other, 2: 2dT, 3: 2Z),
// loaded by that lane alone.  The p3 conversion's products stay on their
// positions (0: X, 1: Y, 2: Z, 3: T); positions 0/1 form Y +- X from two
// quad_perm reads, 2/3 read T / Z directly.
OURO_FI ge_p1p1 ge_add_own_quad(const ge_p1p1& t, const fe& b, bool neg) {
  const fe pa = fe_sel_lanes(t.T, fe_sel_lanes(t.Z, t.X, kQuadHigh), kQuadOdd);
  const fe pb = fe_sel_lanes(fe_sel_lanes(t.X, t.Z, kQuadHigh), t.Y, kQuadOdd);
  const fe m = fe_mul(pa, pb);
  fe u, v;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    // quad_perm [1,1,3,2]: Y, Y, T, Z; [0,0,0,0]: X
    u.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)m.v[i], 0xb5, 0xf, 0xf, true);
    v.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)m.v[i], 0x00, 0xf, 0xf, true);
  }
  const fe a = fe_sel_lanes(fe_sel_lanes(fe_add(u, v), fe_sub(u, v), kQuadOdd), u, kQuadHigh);
  const fe4 g = fe_quad_gather(fe_mul(a, b));
  const fe &A = g.v[0], &B = g.v[1], &C = g.v[2], &D = g.v[3];
  const fe Dp = fe_add(D, C), Dm = fe_sub(D, C);
  ge_p1p1 r;
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_select(Dm, Dp, neg);
  r.T = fe_select(Dp, Dm, neg);
  return r;
}
#endif

OURO_FI ge_p3 ge_p3_add(const ge_p3& p, const ge_p3& q) {
  return ge_p1p1_to_p3(ge_add_cached(p, ge_p3_to_cached(q), false));
}

// P + Q in projective (X:Y:Z) coordinates, complete for a = -1 and non-square
// d (Bernstein-Birkner-Joye-Lange-Peters 2008, "add-2008-bbjlp"):
//   A = Z1 Z2, B = A^2, C = X1 X2, D = Y1 Y2, E = d C D, F = B - E, G = B + E,
//   X3 = A F ((X1 + Y1)(X2 + Y2) - C - D), Y3 = A G (D + C), Z3 = F G.
OURO_FI ge_p2 ge_p2_add(const ge_p2& p, const ge_p2& q) {
  fe A = fe_mul(p.Z, q.Z);
  fe B = fe_sq(A);
  fe C = fe_mul(p.X, q.X);
  fe D = fe_mul(p.Y, q.Y);
  fe E = fe_mul(fe_mul(C, D), fe_d());
  fe F = fe_carry(fe_sub(B, E));
  fe G = fe_carry(fe_add(B, E));
  fe S = fe_mul(fe_carry(fe_add(p.X, p.Y)), fe_carry(fe_add(q.X, q.Y)));
  fe CD = fe_carry(fe_add(C, D));
  fe X3 = fe_mul(fe_mul(A, F), fe_carry(fe_sub(S, CD)));
  fe Y3 = fe_mul(fe_mul(A, G), CD);
  return ge_p2{X3, Y3, fe_mul(F, G)};
}

OURO_FI ge_p3 ge_p3_neg(const ge_p3& p) { return ge_p3{fe_neg(p.X), p.Y, p.Z, fe_neg(p.T)}; }

// [8]P
OURO_FI ge_p3 ge_mul8(const ge_p3& p) {
  ge_p2 t = ge_p1p1_to_p2(ge_p3_dbl(p));
  t = ge_p1p1_to_p2(ge_p2_dbl(t));
  return ge_p1p1_to_p3(ge_p2_dbl(t));
}

// canonical encoding given 1/Z
OURO_FI void ge_encode_with_inv(uint32_t out[8], const fe& X, const fe& Y, const fe& zinv) {
  fe x = fe_mul(X, zinv);
  fe y = fe_mul(Y, zinv);
  uint32_t xw[8];
  fe_to_words(out, y);
  fe_to_words(xw, x);
  out[7] ^= (xw[0] & 1u) << 31;
}

OURO_FI void ge_p2_encode(uint32_t out[8], const ge_p2& p) {
  ge_encode_with_inv(out, p.X, p.Y, fe_invert_vartime(p.Z));
}

// ---- decoding & acceptance predicates (libsodium 1.0.18) -------------------

// ge25519_frombytes (negate = false) / ge25519_frombytes_negate_vartime
// (negate = true).  y is read mod 2^255; x = 0 with the sign bit set is
// accepted.  Returns false when (y^2 - 1)/(d y^2 + 1) is not a square.
// Split around its exponentiation (the latency mode's wave-wide cores run
// that on the wave, wide_cores.h): ge_decode_pre returns u v^7, ge_decode_post
// takes (u v^7)^((p-5)/8).
struct DecodePre { fe y, u, v, v3; };
OURO_FI fe ge_decode_pre(DecodePre& d, const uint32_t s[8]) {
  const fe one = fe_one();
  d.y = fe_from_words(s);
  fe u = fe_sq(d.y);
  fe v = fe_mul(u, fe_d());
  d.u = fe_sub(u, one);  // y^2 - 1
  d.v = fe_add(v, one);  // d y^2 + 1
  d.v3 = fe_mul(fe_sq(d.v), d.v);
  return fe_mul(fe_mul(fe_sq(d.v3), d.v), d.u);  // u v^7
}
OURO_FI bool ge_decode_post(ge_p3* h, const DecodePre& d, const fe& pw, const uint32_t s[8],
                            bool negate) {
  const fe one = fe_one();
  const fe y = d.y, u = d.u, v = d.v;
  fe x = fe_mul(fe_mul(pw, d.v3), u);  // u v^3 (u v^7)^((p-5)/8)
  fe vxx = fe_mul(fe_sq(x), v);
  bool m_root = fe_iszero(fe_sub4(vxx, u));
  bool p_root = fe_iszero(fe_add(vxx, u));
  x = fe_select(x, fe_mul(x, fe_sqrtm1()), m_root);
  const bool sign = (s[7] >> 31) != 0;
  const bool flip = negate ? (fe_isnegative(x) == sign) : (fe_isnegative(x) != sign);
  x = fe_select(fe_neg(x), x, flip);
  h->X = x;
  h->Y = y;
  h->Z = one;
  h->T = fe_mul(x, y);
  return m_root || p_root;
}

OURO_FI bool ge_decode(ge_p3* h, const uint32_t s[8], bool negate) {
  const fe one = fe_one();
  fe y = fe_from_words(s);
  fe u = fe_sq(y);
  fe v = fe_mul(u, fe_d());
  u = fe_sub(u, one);  // y^2 - 1
  v = fe_add(v, one);  // d y^2 + 1
  fe v3 = fe_mul(fe_sq(v), v);
  fe x = fe_mul(fe_mul(fe_sq(v3), v), u);  // u v^7
  x = fe_pow22523(x);
  x = fe_mul(fe_mul(x, v3), u);  // u v^3 (u v^7)^((p-5)/8)
  fe vxx = fe_mul(fe_sq(x), v);
  bool m_root = fe_iszero(fe_sub4(vxx, u));
  bool p_root = fe_iszero(fe_add(vxx, u));
  x = fe_select(x, fe_mul(x, fe_sqrtm1()), m_root);
  const bool sign = (s[7] >> 31) != 0;
  const bool flip = negate ? (fe_isnegative(x) == sign) : (fe_isnegative(x) != sign);
  x = fe_select(fe_neg(x), x, flip);
  h->X = x;
  h->Y = y;
  h->Z = one;
  h->T = fe_mul(x, y);
  return m_root || p_root;
}

// Two decodes on one lane with their exponentiations paired
// (fe_pow22523_x2): same semantics as two ge_decode calls.
#ifndef OURO_DECODE_PAIR
#define OURO_DECODE_PAIR 0  // A/B: 1 pairs the exponentiations (r03c: hdr 70.90 -> 71.25 ms, Ed 12.20 -> 12.33)
#endif
OURO_FI void ge_decode_pair(ge_p3* a, bool* oka, ge_p3* b, bool* okb, const uint32_t sa[8],
                            const uint32_t sb[8], bool negate) {
#if OURO_DECODE_PAIR
  DecodePre pa, pb;
  const fe za = ge_decode_pre(pa, sa), zb = ge_decode_pre(pb, sb);
  const fe_pair pw = fe_pow22523_x2(za, zb);
  *oka = ge_decode_post(a, pa, pw.a, sa, negate);
  *okb = ge_decode_post(b, pb, pw.b, sb, negate);
#else
  *oka = ge_decode(a, sa, negate);
  *okb = ge_decode(b, sb, negate);
#endif
}

// Two decodes at once on a lane quad (latency mode): quad positions 0/2
// decode sa, 1/3 decode sb -- one exponentiation's time instead of two --
// and every lane reads both results.  Same semantics as two ge_decode calls.
OURO_FI void ge_decode_pair_quad(ge_p3* a, bool* oka, ge_p3* b, bool* okb, const uint32_t sa[8],
                                 const uint32_t sb[8], bool negate) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(w[i]) : "v"(sa[i]), "v"(sb[i]), "s"(kQuadOdd));
  ge_p3 P;
  const uint32_t ok = ge_decode(&P, w, negate) ? 1u : 0u;
  *a = ge_p3{fe_quad_bcast<0>(P.X), fe_quad_bcast<0>(P.Y), fe_quad_bcast<0>(P.Z),
             fe_quad_bcast<0>(P.T)};
  *b = ge_p3{fe_quad_bcast<1>(P.X), fe_quad_bcast<1>(P.Y), fe_quad_bcast<1>(P.Z),
             fe_quad_bcast<1>(P.T)};
  *oka = __builtin_amdgcn_mov_dpp((int)ok, 0x00, 0xf, 0xf, true) != 0;
  *okb = __builtin_amdgcn_mov_dpp((int)ok, 0x55, 0xf, 0xf, true) != 0;
#else
  *oka = ge_decode(a, sa, negate);
  *okb = ge_decode(b, sb, negate);
#endif
}

// ge25519_is_canonical: y (bit 255 masked) < p
OURO_FI bool ge_is_canonical(const uint32_t s[8]) {
  bool top_all_ones = (s[7] & 0x7fffffffu) == 0x7fffffffu;
#pragma unroll
  for (int i = 1; i < 7; i++) top_all_ones = top_all_ones && (s[i] == 0xffffffffu);
  return !(top_all_ones && s[0] >= 0xffffffedu);
}

// ge25519_has_small_order: y (sign bit masked) in the 7-entry blocklist
// {0, 1, y8, -y8, p-1, p, p+1}, y8 the order-8 y coordinate.
OURO_FI bool ge_has_small_order(const uint32_t s[8]) {
  const uint32_t top = s[7] & 0x7fffffffu;
  bool mid_zero = true, mid_ones = true;
#pragma unroll
  for (int i = 1; i < 7; i++) {
    mid_zero = mid_zero && s[i] == 0;
    mid_ones = mid_ones && s[i] == 0xffffffffu;
  }
  bool small = (mid_zero && top == 0 && (s[0] == 0 || s[0] == 1)) ||
               (mid_ones && top == 0x7fffffffu &&
                (s[0] == 0xffffffecu || s[0] == 0xffffffedu || s[0] == 0xffffffeeu));
  // y8 = 0x05fc536d...b2c28f95e826 (LE words below), -y8 = p - y8
  const uint32_t y8[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                          0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t ny8[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                           0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  bool e1 = top == y8[7], e2 = top == ny8[7];
#pragma unroll
  for (int i = 0; i < 7; i++) {
    e1 = e1 && s[i] == y8[i];
    e2 = e2 && s[i] == ny8[i];
  }
  return small || e1 || e2;
}

}  // namespace ouro
