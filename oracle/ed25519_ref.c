/*
 * ed25519_ref.c -- CPU restatement of ed25519-dalek 1.0.1 / curve25519-dalek
 * 3.x verification semantics.  TEST INFRASTRUCTURE ONLY (see ntoracle.h).
 *
 * Field: GF(2^255-19) in radix 2^51 (5 x u64, u128 products), the same
 * representation as curve25519-dalek's u64 backend, so that it doubles as
 * the "dalek-equivalent CPU restatement" baseline of BASELINE.md §2.
 *
 * Semantics followed (restated from the pinned crates):
 *   decode s    : reject iff s >= L (incl. bit 255 set)   [ed25519-dalek check_scalar]
 *   decompress  : y = bytes & (2^255-1) NOT reduced/rejected when >= p;
 *                 sqrt_ratio_i(y^2-1, d y^2+1); x := nonneg root, negated by
 *                 the sign bit (x = 0 with sign bit set accepted)
 *   verify_strict (crypto/src/lib.rs:200-204 -> dalek PublicKey::verify_strict):
 *                 s ok, R decodes, A decodes, R and A not small order,
 *                 k = SHA-512(R_bytes||A_bytes||M) mod L,
 *                 accept iff [s]B + [k](-A) == R as points (projective compare)
 *   verify_batch (crypto/src/lib.rs:206-219 -> dalek verify_batch):
 *                 per i in order: s_i ok and A_i decodes (else Err), then
 *                 R_i decodes, then the deterministic rule of Appendix A.3:
 *                 accept iff every R_i == [s_i]B - [k_i]A_i (cofactorless).
 */
#include "ntoracle.h"
#include <string.h>
#include <pthread.h>
#include <stdlib.h>

typedef unsigned __int128 u128;
#define MASK51 ((((uint64_t)1) << 51) - 1)

/* ======================================================================== */
/*  Field arithmetic mod p = 2^255 - 19                                       */
/* ======================================================================== */
typedef struct { uint64_t v[5]; } fe;

static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_copy(fe *h, const fe *f) { *h = *f; }

static void fe_carry(fe *h) {
  uint64_t c;
  for (int pass = 0; pass < 2; ++pass) {
    c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
    c = h->v[1] >> 51; h->v[1] &= MASK51; h->v[2] += c;
    c = h->v[2] >> 51; h->v[2] &= MASK51; h->v[3] += c;
    c = h->v[3] >> 51; h->v[3] &= MASK51; h->v[4] += c;
    c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += 19 * c;
  }
}

/* One weak reduction pass (curve25519-dalek FieldElement51::reduce): every
 * carry is taken from the input limbs, then added once; limbs < 2^52 after. */
static void fe_reduce(fe *h) {
  const uint64_t c0 = h->v[0] >> 51, c1 = h->v[1] >> 51, c2 = h->v[2] >> 51, c3 = h->v[3] >> 51,
                 c4 = h->v[4] >> 51;
  h->v[0] = (h->v[0] & MASK51) + 19 * c4;
  h->v[1] = (h->v[1] & MASK51) + c0;
  h->v[2] = (h->v[2] & MASK51) + c1;
  h->v[3] = (h->v[3] & MASK51) + c2;
  h->v[4] = (h->v[4] & MASK51) + c3;
}

/* Lazy addition as in dalek (no reduction): inputs are mul/sq/sub outputs
 * (limbs < 2^52) or sums of two of them; every consumer (mul/sq: limbs < 2^54,
 * sub: g < 16p limbwise, tobytes: two carry passes) accepts limbs < 2^54. */
static void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
}

/* h = f + 16p - g, one weak reduction (dalek Sub for FieldElement51). */
static void fe_sub(fe *h, const fe *f, const fe *g) {
  static const uint64_t p16_0 = 16 * (MASK51 - 18), p16_i = 16 * MASK51;
  h->v[0] = f->v[0] + p16_0 - g->v[0];
  for (int i = 1; i < 5; ++i) h->v[i] = f->v[i] + p16_i - g->v[i];
  fe_reduce(h);
}

static void fe_neg(fe *h, const fe *f) {
  fe z;
  fe_0(&z);
  fe_sub(h, &z, f);
}

static void fe_mul(fe *h, const fe *f, const fe *g) {
  const uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  const uint64_t g0 = g->v[0], g1 = g->v[1], g2 = g->v[2], g3 = g->v[3], g4 = g->v[4];
  const uint64_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4;
  u128 t0 = (u128)f0 * g0 + (u128)f1 * g4_19 + (u128)f2 * g3_19 + (u128)f3 * g2_19 + (u128)f4 * g1_19;
  u128 t1 = (u128)f0 * g1 + (u128)f1 * g0 + (u128)f2 * g4_19 + (u128)f3 * g3_19 + (u128)f4 * g2_19;
  u128 t2 = (u128)f0 * g2 + (u128)f1 * g1 + (u128)f2 * g0 + (u128)f3 * g4_19 + (u128)f4 * g3_19;
  u128 t3 = (u128)f0 * g3 + (u128)f1 * g2 + (u128)f2 * g1 + (u128)f3 * g0 + (u128)f4 * g4_19;
  u128 t4 = (u128)f0 * g4 + (u128)f1 * g3 + (u128)f2 * g2 + (u128)f3 * g1 + (u128)f4 * g0;
  t1 += (uint64_t)(t0 >> 51);
  t2 += (uint64_t)(t1 >> 51);
  t3 += (uint64_t)(t2 >> 51);
  t4 += (uint64_t)(t3 >> 51);
  uint64_t c = (uint64_t)(t4 >> 51);
  h->v[0] = ((uint64_t)t0 & MASK51) + 19 * c;
  h->v[1] = (uint64_t)t1 & MASK51;
  h->v[2] = (uint64_t)t2 & MASK51;
  h->v[3] = (uint64_t)t3 & MASK51;
  h->v[4] = (uint64_t)t4 & MASK51;
  c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
}

/* Dedicated squaring (15 products instead of 25), as dalek's pow2k. */
static void fe_sq(fe *h, const fe *f) {
  const uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  const uint64_t f0_2 = 2 * f0, f1_2 = 2 * f1, f1_38 = 38 * f1, f2_38 = 38 * f2, f3_38 = 38 * f3;
  const uint64_t f3_19 = 19 * f3, f4_19 = 19 * f4;
  u128 t0 = (u128)f0 * f0 + (u128)f1_38 * f4 + (u128)f2_38 * f3;
  u128 t1 = (u128)f0_2 * f1 + (u128)f2_38 * f4 + (u128)f3_19 * f3;
  u128 t2 = (u128)f0_2 * f2 + (u128)f1 * f1 + (u128)f3_38 * f4;
  u128 t3 = (u128)f0_2 * f3 + (u128)f1_2 * f2 + (u128)f4_19 * f4;
  u128 t4 = (u128)f0_2 * f4 + (u128)f1_2 * f3 + (u128)f2 * f2;
  t1 += (uint64_t)(t0 >> 51);
  t2 += (uint64_t)(t1 >> 51);
  t3 += (uint64_t)(t2 >> 51);
  t4 += (uint64_t)(t3 >> 51);
  uint64_t c = (uint64_t)(t4 >> 51);
  h->v[0] = ((uint64_t)t0 & MASK51) + 19 * c;
  h->v[1] = (uint64_t)t1 & MASK51;
  h->v[2] = (uint64_t)t2 & MASK51;
  h->v[3] = (uint64_t)t3 & MASK51;
  h->v[4] = (uint64_t)t4 & MASK51;
  c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
}

static void fe_sqn(fe *h, const fe *f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

/* little-endian 255-bit load (bit 255 ignored, value NOT reduced mod p) */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    w[i] = 0;
    for (int j = 7; j >= 0; --j) w[i] = (w[i] << 8) | s[8 * i + j];
  }
  h->v[0] = w[0] & MASK51;
  h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  h->v[4] = (w[3] >> 12) & MASK51;
}

/* canonical little-endian encoding (fully reduced mod p) */
static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe h = *f;
  fe_carry(&h);
  /* now h < 2^255 + small; subtract p if h >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= MASK51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= MASK51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= MASK51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= MASK51; h.v[4] += c;
  h.v[4] &= MASK51;
  uint64_t w[4];
  w[0] = h.v[0] | (h.v[1] << 51);
  w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
  w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
  w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int fe_iszero(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  uint8_t acc = 0;
  for (int i = 0; i < 32; ++i) acc |= s[i];
  return acc == 0;
}

static int fe_eq(const fe *f, const fe *g) {
  uint8_t a[32], b[32];
  fe_tobytes(a, f);
  fe_tobytes(b, g);
  return memcmp(a, b, 32) == 0;
}

static int fe_isnegative(const fe *f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  return s[0] & 1;
}

/* z^(2^252 - 3) */
static void fe_pow22523(fe *out, const fe *z) {
  fe t0, t1, t2;
  fe_sq(&t0, z);                 /* 2 */
  fe_sqn(&t1, &t0, 2);           /* 8 */
  fe_mul(&t1, z, &t1);           /* 9 */
  fe_mul(&t0, &t0, &t1);         /* 11 */
  fe_sq(&t0, &t0);               /* 22 */
  fe_mul(&t0, &t1, &t0);         /* 31 = 2^5 - 1 */
  fe_sqn(&t1, &t0, 5);
  fe_mul(&t0, &t1, &t0);         /* 2^10 - 1 */
  fe_sqn(&t1, &t0, 10);
  fe_mul(&t1, &t1, &t0);         /* 2^20 - 1 */
  fe_sqn(&t2, &t1, 20);
  fe_mul(&t1, &t2, &t1);         /* 2^40 - 1 */
  fe_sqn(&t1, &t1, 10);
  fe_mul(&t0, &t1, &t0);         /* 2^50 - 1 */
  fe_sqn(&t1, &t0, 50);
  fe_mul(&t1, &t1, &t0);         /* 2^100 - 1 */
  fe_sqn(&t2, &t1, 100);
  fe_mul(&t1, &t2, &t1);         /* 2^200 - 1 */
  fe_sqn(&t1, &t1, 50);
  fe_mul(&t0, &t1, &t0);         /* 2^250 - 1 */
  fe_sqn(&t0, &t0, 2);           /* 2^252 - 4 */
  fe_mul(out, &t0, z);           /* 2^252 - 3 */
}

/* z^(p-2) = z^(2^255 - 21) */
static void fe_invert(fe *out, const fe *z) {
  fe t0, t1, t2, t3;
  fe_sq(&t0, z);                 /* 2 */
  fe_sqn(&t1, &t0, 2);           /* 8 */
  fe_mul(&t1, z, &t1);           /* 9 */
  fe_mul(&t0, &t0, &t1);         /* 11 */
  fe_sq(&t2, &t0);               /* 22 */
  fe_mul(&t1, &t1, &t2);         /* 31 */
  fe_sqn(&t2, &t1, 5);
  fe_mul(&t1, &t2, &t1);         /* 2^10 - 1 */
  fe_sqn(&t2, &t1, 10);
  fe_mul(&t2, &t2, &t1);         /* 2^20 - 1 */
  fe_sqn(&t3, &t2, 20);
  fe_mul(&t2, &t3, &t2);         /* 2^40 - 1 */
  fe_sqn(&t2, &t2, 10);
  fe_mul(&t1, &t2, &t1);         /* 2^50 - 1 */
  fe_sqn(&t2, &t1, 50);
  fe_mul(&t2, &t2, &t1);         /* 2^100 - 1 */
  fe_sqn(&t3, &t2, 100);
  fe_mul(&t2, &t3, &t2);         /* 2^200 - 1 */
  fe_sqn(&t2, &t2, 50);
  fe_mul(&t1, &t2, &t1);         /* 2^250 - 1 */
  fe_sqn(&t1, &t1, 5);           /* 2^255 - 32 */
  fe_mul(out, &t1, &t0);         /* 2^255 - 21 */
}

/* ======================================================================== */
/*  Curve constants (derived at init, not transcribed)                        */
/* ======================================================================== */
static fe C_D, C_D2, C_SQRTM1;
static int consts_ready = 0;
static pthread_once_t consts_once = PTHREAD_ONCE_INIT;

/* ======================================================================== */
/*  Points: extended (X:Y:Z:T), completed (E,F,G,H), cached, affine-niels     */
/* ======================================================================== */
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe E, F, G, H; } ge_p1p1;              /* X=EF Y=GH Z=FG T=EH */
typedef struct { fe YpX, YmX, Z2, T2d; } ge_cached;     /* (Y+X, Y-X, 2Z, 2dT) */
typedef struct { fe ypx, ymx, xy2d; } ge_niels;         /* affine (y+x, y-x, 2dxy) */

static void ge_p3_0(ge_p3 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); fe_0(&h->T); }
static void ge_p2_0(ge_p2 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); }

static void p1p1_to_p2(ge_p2 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->E, &p->F);
  fe_mul(&r->Y, &p->G, &p->H);
  fe_mul(&r->Z, &p->F, &p->G);
}
static void p1p1_to_p3(ge_p3 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->E, &p->F);
  fe_mul(&r->Y, &p->G, &p->H);
  fe_mul(&r->Z, &p->F, &p->G);
  fe_mul(&r->T, &p->E, &p->H);
}
static void p3_to_p2(ge_p2 *r, const ge_p3 *p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }

static void p3_to_cached(ge_cached *r, const ge_p3 *p) {
  fe_add(&r->YpX, &p->Y, &p->X);
  fe_sub(&r->YmX, &p->Y, &p->X);
  fe_add(&r->Z2, &p->Z, &p->Z);
  fe_mul(&r->T2d, &p->T, &C_D2);
}

/* doubling of (X:Y:Z) for a = -1 (dbl-2008-hwcd) */
static void ge_dbl(ge_p1p1 *r, const ge_p2 *p) {
  fe A, B, C, S;
  fe_sq(&A, &p->X);
  fe_sq(&B, &p->Y);
  fe_sq(&C, &p->Z);
  fe_add(&C, &C, &C);
  fe_add(&S, &p->X, &p->Y);
  fe_sq(&S, &S);
  fe_sub(&r->G, &B, &A);          /* G = B - A   (D + B, D = -A) */
  fe_add(&r->H, &A, &B);
  fe_neg(&r->H, &r->H);           /* H = -A - B  (D - B) */
  fe_sub(&r->E, &S, &A);
  fe_sub(&r->E, &r->E, &B);       /* E = (X+Y)^2 - A - B */
  fe_sub(&r->F, &r->G, &C);       /* F = G - C */
}

static void ge_add_cached(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q, int neg) {
  fe A, B, C, D, t;
  fe_sub(&t, &p->Y, &p->X);
  fe_mul(&A, &t, neg ? &q->YpX : &q->YmX);
  fe_add(&t, &p->Y, &p->X);
  fe_mul(&B, &t, neg ? &q->YmX : &q->YpX);
  fe_mul(&C, &p->T, &q->T2d);
  if (neg) fe_neg(&C, &C);
  fe_mul(&D, &p->Z, &q->Z2);
  fe_sub(&r->E, &B, &A);
  fe_sub(&r->F, &D, &C);
  fe_add(&r->G, &D, &C);
  fe_add(&r->H, &B, &A);
}

static void ge_add_niels(ge_p1p1 *r, const ge_p3 *p, const ge_niels *q, int neg) {
  fe A, B, C, D, t;
  fe_sub(&t, &p->Y, &p->X);
  fe_mul(&A, &t, neg ? &q->ypx : &q->ymx);
  fe_add(&t, &p->Y, &p->X);
  fe_mul(&B, &t, neg ? &q->ymx : &q->ypx);
  fe_mul(&C, &p->T, &q->xy2d);
  if (neg) fe_neg(&C, &C);
  fe_add(&D, &p->Z, &p->Z);
  fe_sub(&r->E, &B, &A);
  fe_sub(&r->F, &D, &C);
  fe_add(&r->G, &D, &C);
  fe_add(&r->H, &B, &A);
}

static void ge_add_p3(ge_p3 *r, const ge_p3 *p, const ge_p3 *q) {
  ge_cached c;
  ge_p1p1 t;
  p3_to_cached(&c, q);
  ge_add_cached(&t, p, &c, 0);
  p1p1_to_p3(r, &t);
}

static void ge_dbl_p3(ge_p3 *r, const ge_p3 *p) {
  ge_p2 q;
  ge_p1p1 t;
  p3_to_p2(&q, p);
  ge_dbl(&t, &q);
  p1p1_to_p3(r, &t);
}

static void ge_neg(ge_p3 *r, const ge_p3 *p) {
  fe_neg(&r->X, &p->X);
  r->Y = p->Y;
  r->Z = p->Z;
  fe_neg(&r->T, &p->T);
}

static void ge_tobytes(uint8_t s[32], const ge_p3 *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

static int ge_is_identity(const ge_p3 *p) {
  return fe_iszero(&p->X) && fe_eq(&p->Y, &p->Z);
}

/* projective equality (curve25519-dalek EdwardsPoint::ct_eq) */
static int ge_eq_proj(const fe *X1, const fe *Y1, const fe *Z1, const fe *X2, const fe *Y2,
                      const fe *Z2) {
  fe a, b, c, d;
  fe_mul(&a, X1, Z2);
  fe_mul(&b, X2, Z1);
  fe_mul(&c, Y1, Z2);
  fe_mul(&d, Y2, Z1);
  return fe_eq(&a, &b) && fe_eq(&c, &d);
}

/* sqrt_ratio_i(u, v): returns 1 iff u/v is a nonzero square or u == 0;
 * r = nonnegative root (curve25519-dalek field.rs semantics). */
static int fe_sqrt_ratio_i(fe *r, const fe *u, const fe *v) {
  fe v3, v7, t, check, negu, negu_i;
  fe_sq(&v3, v);
  fe_mul(&v3, &v3, v);            /* v^3 */
  fe_sq(&v7, &v3);
  fe_mul(&v7, &v7, v);            /* v^7 */
  fe_mul(&t, u, &v7);
  fe_pow22523(&t, &t);            /* (u v^7)^((p-5)/8) */
  fe_mul(&t, &t, &v3);
  fe_mul(r, &t, u);               /* r = u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&check, r);
  fe_mul(&check, &check, v);      /* v r^2 */
  fe_neg(&negu, u);
  fe_mul(&negu_i, &negu, &C_SQRTM1);
  int correct = fe_eq(&check, u);
  int flipped = fe_eq(&check, &negu);
  int flipped_i = fe_eq(&check, &negu_i);
  if (flipped || flipped_i) fe_mul(r, r, &C_SQRTM1);
  if (fe_isnegative(r)) fe_neg(r, r);
  return correct || flipped;
}

/* CompressedEdwardsY::decompress */
static int ge_frombytes(ge_p3 *h, const uint8_t s[32]) {
  fe u, v, yy;
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&yy, &h->Y);
  fe_sub(&u, &yy, &h->Z);
  fe_mul(&v, &yy, &C_D);
  fe_add(&v, &v, &h->Z);
  if (!fe_sqrt_ratio_i(&h->X, &u, &v)) return 0;
  if (s[31] >> 7) fe_neg(&h->X, &h->X);
  fe_mul(&h->T, &h->X, &h->Y);
  return 1;
}

static int ge_is_small_order(const ge_p3 *p) {
  ge_p3 t;
  ge_dbl_p3(&t, p);
  ge_dbl_p3(&t, &t);
  ge_dbl_p3(&t, &t);
  return ge_is_identity(&t);
}

/* ======================================================================== */
/*  Scalars mod L = 2^252 + 27742317777372353535851937790883648493            */
/* ======================================================================== */
/* Generic little-endian u32 bignum helpers (small sizes, clarity first). */
static const uint32_t L_W[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                0x00000000u, 0x00000000u, 0x00000000u, 0x10000000u};
static uint32_t MU_W[9]; /* floor(2^512 / L), 253 bits -> 8 words + 1 */

static void bn_mul(uint32_t *out, const uint32_t *a, int na, const uint32_t *b, int nb) {
  memset(out, 0, sizeof(uint32_t) * (na + nb));
  for (int i = 0; i < na; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < nb; ++j) {
      uint64_t t = (uint64_t)a[i] * b[j] + out[i + j] + c;
      out[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    out[i + nb] = (uint32_t)c;
  }
}

/* a >= b ? (n words) */
static int bn_ge(const uint32_t *a, const uint32_t *b, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}
static void bn_sub(uint32_t *a, const uint32_t *b, int n) { /* a -= b, mod 2^(32n) */
  int64_t br = 0;
  for (int i = 0; i < n; ++i) {
    int64_t t = (int64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)t;
    br = t < 0;
  }
}

static void compute_mu(void) {
  /* long division of 2^512 by L (shift-subtract), result < 2^260 */
  uint32_t rem[17], q[17];
  memset(rem, 0, sizeof rem);
  memset(q, 0, sizeof q);
  uint32_t Lx[17];
  memset(Lx, 0, sizeof Lx);
  memcpy(Lx, L_W, sizeof L_W);
  for (int bit = 512; bit >= 0; --bit) {
    /* rem = rem*2 + (bit == 512) */
    for (int i = 16; i > 0; --i) rem[i] = (rem[i] << 1) | (rem[i - 1] >> 31);
    rem[0] = (rem[0] << 1) | (bit == 512 ? 1u : 0u);
    if (bn_ge(rem, Lx, 17)) {
      bn_sub(rem, Lx, 17);
      q[bit / 32] |= 1u << (bit % 32);
    }
  }
  memcpy(MU_W, q, sizeof MU_W);
}

static void load_words(uint32_t *w, const uint8_t *b, int nbytes) {
  for (int i = 0; i < nbytes / 4; ++i)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}
static void store_words(uint8_t *b, const uint32_t *w, int nwords) {
  for (int i = 0; i < nwords; ++i) {
    b[4 * i] = (uint8_t)w[i]; b[4 * i + 1] = (uint8_t)(w[i] >> 8);
    b[4 * i + 2] = (uint8_t)(w[i] >> 16); b[4 * i + 3] = (uint8_t)(w[i] >> 24);
  }
}

/* Barrett reduction (HAC 14.42, b = 2^32, k = 8): x (16 words) mod L */
static void sc_reduce_words(uint32_t out[8], const uint32_t x[16]) {
  uint32_t q1[9], q2[18], r1[9], r2[18];
  memcpy(q1, x + 7, 9 * sizeof(uint32_t));          /* floor(x / b^(k-1)) */
  bn_mul(q2, q1, 9, MU_W, 9);                        /* q1 * mu */
  uint32_t *q3 = q2 + 9;                             /* floor(q2 / b^(k+1)), 9 words */
  memcpy(r1, x, 9 * sizeof(uint32_t));               /* x mod b^(k+1) */
  uint32_t t[18];
  bn_mul(t, q3, 9, L_W, 8);                          /* q3 * L */
  memcpy(r2, t, 9 * sizeof(uint32_t));               /* mod b^(k+1) */
  bn_sub(r1, r2, 9);                                 /* wraps mod b^(k+1) if negative */
  uint32_t L9[9];
  memcpy(L9, L_W, sizeof L_W);
  L9[8] = 0;
  while (bn_ge(r1, L9, 9)) bn_sub(r1, L9, 9);
  memcpy(out, r1, 8 * sizeof(uint32_t));
}

void ntor_sc_reduce64(const uint8_t in64[64], uint8_t out32[32]) {
  uint32_t x[16], r[8];
  load_words(x, in64, 64);
  sc_reduce_words(r, x);
  store_words(out32, r, 8);
}

/* dalek check_scalar: accept iff s < L (bit 255 set -> reject) */
int ntor_sc_is_canonical(const uint8_t s32[32]) {
  if ((s32[31] & 0xf0) == 0) return 1;
  if (s32[31] & 0x80) return 0;
  uint32_t s[8];
  load_words(s, s32, 32);
  return !bn_ge(s, L_W, 8);
}

/* s = (a * b + c) mod L, all 32-byte little-endian (a may be up to 2^256) */
static void sc_muladd(uint8_t s32[32], const uint8_t a32[32], const uint8_t b32[32],
                      const uint8_t c32[32]) {
  uint32_t a[8], b[8], c[8], p[16], r[8];
  load_words(a, a32, 32);
  load_words(b, b32, 32);
  load_words(c, c32, 32);
  bn_mul(p, a, 8, b, 8);
  uint64_t carry = 0;
  for (int i = 0; i < 16; ++i) {
    uint64_t t = (uint64_t)p[i] + (i < 8 ? c[i] : 0) + carry;
    p[i] = (uint32_t)t;
    carry = t >> 32;
  }
  /* a*b + c < 2^512 for a, b < 2^256 - 1 ... guaranteed for our inputs (b < L) */
  sc_reduce_words(r, p);
  store_words(s32, r, 8);
}

/* ======================================================================== */
/*  Scalar multiplication                                                    */
/* ======================================================================== */
/* width-w non-adjacent form of a scalar < 2^255 (digits odd, |d| < 2^(w-1)) */
static void wnaf(int8_t naf[257], const uint8_t s[32], int w) {
  uint64_t x[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i)
    for (int j = 7; j >= 0; --j) x[i] = (x[i] << 8) | s[8 * i + j];
  memset(naf, 0, 257);
  const uint64_t width = 1ULL << w, wmask = width - 1;
  uint64_t carry = 0;
  int pos = 0;
  while (pos < 256) {
    int idx = pos / 64, bit = pos % 64;
    uint64_t buf = x[idx] >> bit;
    if (bit + w > 64 && idx < 4) buf |= x[idx + 1] << (64 - bit);
    uint64_t win = carry + (buf & wmask);
    if ((win & 1) == 0) { pos += 1; continue; }
    if (win < width / 2) { carry = 0; naf[pos] = (int8_t)win; }
    else { carry = 1; naf[pos] = (int8_t)((int64_t)win - (int64_t)width); }
    pos += w;
  }
  if (carry) naf[256] = 1;
}

#define BTAB_W 8
static ge_niels BTAB[1 << (BTAB_W - 2)]; /* odd multiples B, 3B, ..., 127B (affine niels) */
static ge_p3 BASE;

static void p3_to_niels(ge_niels *n, const ge_p3 *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_add(&n->ypx, &y, &x);
  fe_sub(&n->ymx, &y, &x);
  fe_mul(&n->xy2d, &x, &y);
  fe_mul(&n->xy2d, &n->xy2d, &C_D2);
}

static void init_consts(void) {
  fe t, n;
  /* d = -121665 / 121666 */
  fe_0(&t); t.v[0] = 121666;
  fe_invert(&t, &t);
  fe_0(&n); n.v[0] = 121665;
  fe_neg(&n, &n);
  fe_mul(&C_D, &n, &t);
  fe_add(&C_D2, &C_D, &C_D);
  /* sqrt(-1) = 2^((p-1)/4); (p-1)/4 = 2^253 - 5.  2^((p-1)/4) = (2^(2^252-3))^2 * 2^(1) ... */
  /* compute via 2^((p-1)/4) = 2^(2 (2^252 - 3) + 1)  since 2(2^252-3)+1 = 2^253 - 5 */
  fe two;
  fe_0(&two); two.v[0] = 2;
  fe_pow22523(&t, &two);
  fe_sq(&t, &t);
  fe_mul(&C_SQRTM1, &t, &two);
  /* base point: y = 4/5, x even */
  uint8_t bb[32];
  fe four, five;
  fe_0(&four); four.v[0] = 4;
  fe_0(&five); five.v[0] = 5;
  fe_invert(&five, &five);
  fe_mul(&t, &four, &five);
  fe_tobytes(bb, &t);
  ge_frombytes(&BASE, bb);
  /* odd-multiples table of B */
  ge_p3 B2, cur;
  ge_dbl_p3(&B2, &BASE);
  cur = BASE;
  for (int i = 0; i < (1 << (BTAB_W - 2)); ++i) {
    p3_to_niels(&BTAB[i], &cur);
    ge_add_p3(&cur, &cur, &B2);
  }
  compute_mu();
  consts_ready = 1;
}
static void ensure_consts(void) { pthread_once(&consts_once, init_consts); }

/* r = [a]A + [b]B, variable time (dalek vartime_double_scalar_mul_basepoint) */
static void ge_double_scalarmult_vartime(ge_p2 *r, const uint8_t a[32], const ge_p3 *A,
                                         const uint8_t b[32]) {
  int8_t na[257], nb[257];
  wnaf(na, a, 5);
  wnaf(nb, b, BTAB_W);
  ge_cached Ai[8];
  ge_p3 A2, cur;
  ge_dbl_p3(&A2, A);
  cur = *A;
  for (int i = 0; i < 8; ++i) {
    p3_to_cached(&Ai[i], &cur);
    ge_add_p3(&cur, &cur, &A2);
  }
  ge_p2_0(r);
  int i = 256;
  while (i >= 0 && na[i] == 0 && nb[i] == 0) --i;
  ge_p1p1 t;
  ge_p3 u;
  for (; i >= 0; --i) {
    ge_dbl(&t, r);
    if (na[i] > 0) { p1p1_to_p3(&u, &t); ge_add_cached(&t, &u, &Ai[na[i] / 2], 0); }
    else if (na[i] < 0) { p1p1_to_p3(&u, &t); ge_add_cached(&t, &u, &Ai[(-na[i]) / 2], 1); }
    if (nb[i] > 0) { p1p1_to_p3(&u, &t); ge_add_niels(&t, &u, &BTAB[nb[i] / 2], 0); }
    else if (nb[i] < 0) { p1p1_to_p3(&u, &t); ge_add_niels(&t, &u, &BTAB[(-nb[i]) / 2], 1); }
    p1p1_to_p2(r, &t);
  }
}

/* generic [s]P, double-and-add over all 256 bits (oracle helper) */
static void ge_scalarmult(ge_p3 *r, const ge_p3 *P, const uint8_t s[32]) {
  ge_p3_0(r);
  for (int i = 255; i >= 0; --i) {
    ge_dbl_p3(r, r);
    if ((s[i / 8] >> (i % 8)) & 1) ge_add_p3(r, r, P);
  }
}

static void ge_scalarmult_base(ge_p3 *r, const uint8_t s[32]) { ge_scalarmult(r, &BASE, s); }

/* ======================================================================== */
/*  Ed25519                                                                   */
/* ======================================================================== */
static void hash_ram(uint8_t k[32], const uint8_t R[32], const uint8_t A[32], const uint8_t *m,
                     uint64_t len) {
  /* SHA-512(R || A || M) reduced mod L: Scalar::from_hash */
  uint8_t *buf = (uint8_t *)malloc(64 + len);
  memcpy(buf, R, 32);
  memcpy(buf + 32, A, 32);
  if (len) memcpy(buf + 64, m, len);
  uint8_t h[64];
  ntor_sha512(buf, 64 + len, h);
  free(buf);
  ntor_sc_reduce64(h, k);
}

void ntor_ed25519_pubkey(const uint8_t seed32[32], uint8_t pk32[32]) {
  ensure_consts();
  uint8_t h[64];
  ntor_sha512(seed32, 32, h);
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  ge_p3 A;
  ge_scalarmult_base(&A, h);
  ge_tobytes(pk32, &A);
}

void ntor_ed25519_sign(const uint8_t seed32[32], const uint8_t pk32[32], const uint8_t *msg,
                       uint64_t len, uint8_t sig64[64]) {
  ensure_consts();
  uint8_t h[64], r64[64], r[32], k[32];
  ntor_sha512(seed32, 32, h);
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  uint8_t *buf = (uint8_t *)malloc(32 + len);
  memcpy(buf, h + 32, 32);
  if (len) memcpy(buf + 32, msg, len);
  ntor_sha512(buf, 32 + len, r64);
  free(buf);
  ntor_sc_reduce64(r64, r);
  ge_p3 R;
  ge_scalarmult_base(&R, r);
  ge_tobytes(sig64, &R);
  hash_ram(k, sig64, pk32, msg, len);
  sc_muladd(sig64 + 32, k, h, r);
}

/* Shared core: returns 1 iff R == [s]B - [k]A, with decode checks.
 * strict: additionally reject small-order R or A. */
static int verify_core(const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t *msg,
                       uint64_t len, int strict) {
  ensure_consts();
  if (!ntor_sc_is_canonical(sig64 + 32)) return 0;
  ge_p3 A, R;
  if (!ge_frombytes(&A, pk32)) return 0;
  if (!ge_frombytes(&R, sig64)) return 0;
  if (strict && (ge_is_small_order(&R) || ge_is_small_order(&A))) return 0;
  uint8_t k[32];
  hash_ram(k, sig64, pk32, msg, len);
  ge_p3 negA;
  ge_neg(&negA, &A);
  ge_p2 Rp;
  uint8_t s[32];
  memcpy(s, sig64 + 32, 32);
  s[31] &= 0x7f; /* Scalar::from_bits (no-op for accepted s) */
  ge_double_scalarmult_vartime(&Rp, k, &negA, s);
  return ge_eq_proj(&Rp.X, &Rp.Y, &Rp.Z, &R.X, &R.Y, &R.Z);
}

int ntor_ed25519_verify_strict(const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t *msg,
                               uint64_t len) {
  return verify_core(pk32, sig64, msg, len, 1);
}

int ntor_ed25519_verify_cofactorless(const uint8_t pk32[32], const uint8_t sig64[64],
                                     const uint8_t *msg, uint64_t len) {
  return verify_core(pk32, sig64, msg, len, 0);
}

int ntor_ed25519_verify_batch(const uint8_t *pk32, const uint8_t *sig64, uint64_t cnt,
                              const uint8_t *msg, uint64_t len) {
  /* crypto/src/lib.rs:212-217: per entry s check then A decode; first failure -> Err.
   * dalek verify_batch: R decode (in the multiscalar mul), equation (A.3 rule).
   * The decision is the AND of all per-entry checks, so order does not matter. */
  for (uint64_t i = 0; i < cnt; ++i)
    if (!verify_core(pk32 + 32 * i, sig64 + 64 * i, msg, len, 0)) return 0;
  return 1;
}

typedef struct {
  const uint8_t *pk, *sig, *msg;
  const uint64_t *off, *len;
  const uint64_t *first;
  const uint32_t *cnt;
  uint64_t lo, hi;
  uint8_t *res;  /* one byte per item */
  uint8_t *sigres;
  int mode;      /* 0 strict-many, 1 batch-groups */
} vjob;

static void *verify_worker(void *p) {
  vjob *j = (vjob *)p;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    if (j->mode == 0) {
      j->res[i] = (uint8_t)ntor_ed25519_verify_strict(j->pk + 32 * i, j->sig + 64 * i,
                                                      j->msg + j->off[i], j->len[i]);
    } else {
      int ok = 1;
      for (uint32_t t = 0; t < j->cnt[i]; ++t) {
        uint64_t e = j->first[i] + t;
        int v = verify_core(j->pk + 32 * e, j->sig + 64 * e, j->msg + 32 * i, 32, 0);
        if (j->sigres) j->sigres[e] = (uint8_t)v;
        ok &= v;
      }
      j->res[i] = (uint8_t)ok;
    }
  }
  return NULL;
}

static void run_pool(vjob *tmpl, uint64_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t th[256];
  vjob jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = *tmpl;
    jobs[t].lo = n * t / nthreads;
    jobs[t].hi = n * (t + 1) / nthreads;
    if (nthreads == 1) verify_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void ntor_ed25519_verify_strict_many(const uint8_t *pk32, const uint8_t *sig64, const uint8_t *msg,
                                     const uint64_t *off, const uint64_t *len, uint64_t n,
                                     uint8_t *out_bitmap, int nthreads) {
  ensure_consts();
  uint8_t *res = (uint8_t *)calloc(n ? n : 1, 1);
  vjob j = {pk32, sig64, msg, off, len, NULL, NULL, 0, 0, res, NULL, 0};
  run_pool(&j, n, nthreads);
  memset(out_bitmap, 0, (n + 7) / 8);
  for (uint64_t i = 0; i < n; ++i)
    if (res[i]) out_bitmap[i / 8] |= (uint8_t)(1u << (i % 8));
  free(res);
}

void ntor_ed25519_verify_batch_groups(const uint8_t *pk32, const uint8_t *sig64,
                                      const uint64_t *first, const uint32_t *cnt,
                                      const uint8_t *msg32, uint64_t G, uint8_t *out_group_bitmap,
                                      uint8_t *out_sig_bitmap, int nthreads) {
  ensure_consts();
  uint64_t nsig = 0;
  for (uint64_t g = 0; g < G; ++g)
    if (first[g] + cnt[g] > nsig) nsig = first[g] + cnt[g];
  uint8_t *res = (uint8_t *)calloc(G ? G : 1, 1);
  uint8_t *sres = out_sig_bitmap ? (uint8_t *)calloc(nsig ? nsig : 1, 1) : NULL;
  vjob j = {pk32, sig64, msg32, NULL, NULL, first, cnt, 0, 0, res, sres, 1};
  run_pool(&j, G, nthreads);
  memset(out_group_bitmap, 0, (G + 7) / 8);
  for (uint64_t g = 0; g < G; ++g)
    if (res[g]) out_group_bitmap[g / 8] |= (uint8_t)(1u << (g % 8));
  if (out_sig_bitmap) {
    memset(out_sig_bitmap, 0, (nsig + 7) / 8);
    for (uint64_t e = 0; e < nsig; ++e)
      if (sres[e]) out_sig_bitmap[e / 8] |= (uint8_t)(1u << (e % 8));
    free(sres);
  }
  free(res);
}

/* ======================================================================== */
/*  Diagnostics for the corpus generator                                     */
/* ======================================================================== */
int ntor_point_decodes(const uint8_t p32[32]) {
  ensure_consts();
  ge_p3 P;
  return ge_frombytes(&P, p32);
}

int ntor_point_is_small_order(const uint8_t p32[32]) {
  ensure_consts();
  ge_p3 P;
  if (!ge_frombytes(&P, p32)) return 0;
  return ge_is_small_order(&P);
}

static const uint8_t L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58,
                                    0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
                                    0,    0,    0,    0,    0,    0,    0,    0,
                                    0,    0,    0,    0,    0,    0,    0,    0x10};

static int p3_has_torsion(const ge_p3 *P) {
  ge_p3 t;
  ge_scalarmult(&t, P, L_BYTES);
  return !ge_is_identity(&t);
}

int ntor_point_has_torsion(const uint8_t p32[32]) {
  ensure_consts();
  ge_p3 P;
  if (!ge_frombytes(&P, p32)) return 0;
  return p3_has_torsion(&P);
}

/* 1 iff [L]P != identity is false, i.e. returns 1 when P has a nonzero prime-order part */
static int p3_has_torsion_free_part(const ge_p3 *P) {
  /* P has a nonzero prime-order component iff [8]P != identity */
  ge_p3 t;
  ge_dbl_p3(&t, P);
  ge_dbl_p3(&t, &t);
  ge_dbl_p3(&t, &t);
  return !ge_is_identity(&t);
}

int ntor_ed25519_batch_class(const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t *msg,
                             uint64_t len) {
  ensure_consts();
  if (!ntor_sc_is_canonical(sig64 + 32)) return 0;
  ge_p3 A, R;
  if (!ge_frombytes(&A, pk32) || !ge_frombytes(&R, sig64)) return 0;
  uint8_t k[32];
  hash_ram(k, sig64, pk32, msg, len);
  /* D = R + [k]A - [s]B */
  ge_p3 kA, sB, D, negsB;
  ge_scalarmult(&kA, &A, k);
  uint8_t s[32];
  memcpy(s, sig64 + 32, 32);
  ge_scalarmult_base(&sB, s);
  ge_neg(&negsB, &sB);
  ge_add_p3(&D, &R, &kA);
  ge_add_p3(&D, &D, &negsB);
  int D_zero = ge_is_identity(&D);
  int D_torsion_only = D_zero || !p3_has_torsion_free_part(&D);
  int A_tors = p3_has_torsion(&A);
  if (D_zero && !A_tors) return 1;
  if (!D_torsion_only) return 0;
  return 2;
}

int ntor_point_add(const uint8_t p32[32], const uint8_t q32[32], uint8_t out32[32]) {
  ensure_consts();
  ge_p3 P, Q, S;
  if (!ge_frombytes(&P, p32) || !ge_frombytes(&Q, q32)) return 0;
  ge_add_p3(&S, &P, &Q);
  ge_tobytes(out32, &S);
  return 1;
}

int ntor_point_scalarmul(const uint8_t p32[32], const uint8_t s32[32], uint8_t out32[32]) {
  ensure_consts();
  ge_p3 P, S;
  if (!ge_frombytes(&P, p32)) return 0;
  ge_scalarmult(&S, &P, s32);
  ge_tobytes(out32, &S);
  return 1;
}

void ntor_basepoint_mul(const uint8_t s32[32], uint8_t out32[32]) {
  ensure_consts();
  ge_p3 S;
  ge_scalarmult_base(&S, s32);
  ge_tobytes(out32, &S);
}

void ntor_torsion_point(int i, uint8_t out32[32]) {
  ensure_consts();
  /* T8 = [L] P for a point P with full torsion: try y = 2, 3, ... until [L]P has order 8 */
  static ge_p3 T8;
  static int have = 0;
  if (!have) {
    for (uint64_t y = 2;; ++y) {
      uint8_t enc[32] = {0};
      enc[0] = (uint8_t)y;
      ge_p3 P, t;
      if (!ge_frombytes(&P, enc)) continue;
      ge_scalarmult(&t, &P, L_BYTES);
      ge_p3 t4 = t;
      ge_dbl_p3(&t4, &t4);
      ge_dbl_p3(&t4, &t4);
      if (ge_is_identity(&t4)) continue; /* order < 8 */
      T8 = t;
      have = 1;
      break;
    }
  }
  ge_p3 r;
  ge_p3_0(&r);
  for (int k = 0; k < (i & 7); ++k) ge_add_p3(&r, &r, &T8);
  ge_tobytes(out32, &r);
}

/* ======================================================================== */
/*  dalek's verify_batch as dalek computes it (CPU BASELINE ONLY)            */
/* ======================================================================== */
/* ed25519-dalek 1.0.1 verify_batch (crypto/src/lib.rs:218): random 128-bit z_i,
 * one vartime multiscalar multiplication
 *     [-sum z_i s_i]B + sum [z_i]R_i + sum [z_i k_i]A_i  ==  identity ?
 * by Straus with width-5 NAF digits and per-point tables of odd multiples
 * (curve25519-dalek's VartimeMultiscalarMul below 190 points).  This is the
 * timing restatement behind bench.py's config-3 CPU baseline: the parity
 * checker for batches stays ntor_ed25519_verify_batch (the deterministic
 * rule of SURVEY A.3); both agree except on dalek's random class.
 * z_i come from ChaCha20 keyed by `zkey` (stream = entry index) instead of
 * merlin + thread_rng: the decision does not depend on which z are drawn
 * outside that class. */
int ntor_ed25519_verify_batch_dalek(const uint8_t *pk32, const uint8_t *sig64, uint64_t cnt,
                                    const uint8_t *msg, uint64_t len, const uint8_t zkey[32]) {
  ensure_consts();
  if (cnt == 0) return 1;
  const uint64_t npts = 2 * cnt + 1;
  ge_p3 *pts = (ge_p3 *)malloc(npts * sizeof(ge_p3));
  uint8_t *sc = (uint8_t *)calloc(npts, 32);
  ge_cached *tab = (ge_cached *)malloc(npts * 8 * sizeof(ge_cached));
  int8_t *naf = (int8_t *)malloc(npts * 257);
  int ok = 1;
  /* crypto/src/lib.rs:212-217: s check and A decode per entry, first failure -> Err */
  for (uint64_t i = 0; i < cnt && ok; ++i) {
    if (!ntor_sc_is_canonical(sig64 + 64 * i + 32) || !ge_frombytes(&pts[1 + cnt + i], pk32 + 32 * i)) ok = 0;
  }
  for (uint64_t i = 0; i < cnt && ok; ++i)
    if (!ge_frombytes(&pts[1 + i], sig64 + 64 * i)) ok = 0;  /* R decompress */
  if (ok) {
    uint8_t zero[32] = {0}, bco[32] = {0};
    pts[0] = BASE;
    for (uint64_t i = 0; i < cnt; ++i) {
      uint8_t z[32] = {0}, k[32];
      ntor_chacha20_keystream(zkey, i, 0, z, 16);           /* 128-bit z_i */
      memcpy(sc + 32 * (1 + i), z, 32);                     /* R_i: z_i */
      hash_ram(k, sig64 + 64 * i, pk32 + 32 * i, msg, len);
      sc_muladd(sc + 32 * (1 + cnt + i), z, k, zero);       /* A_i: z_i k_i mod L */
      sc_muladd(bco, z, sig64 + 64 * i + 32, bco);          /* sum z_i s_i mod L */
    }
    /* B: L - bco (mod L) */
    uint32_t l[8], b[8];
    load_words(b, bco, 32);
    memcpy(l, L_W, sizeof l);
    int nz = 0;
    for (int q = 0; q < 8; ++q) nz |= b[q] != 0;
    if (nz) bn_sub(l, b, 8);
    else memset(l, 0, sizeof l);
    store_words(sc, l, 8);
    for (uint64_t j = 0; j < npts; ++j) {
      wnaf(naf + 257 * j, sc + 32 * j, 5);
      ge_p3 P2, cur = pts[j];
      ge_dbl_p3(&P2, &pts[j]);
      for (int q = 0; q < 8; ++q) {  /* P, 3P, ..., 15P */
        p3_to_cached(&tab[8 * j + q], &cur);
        if (q < 7) ge_add_p3(&cur, &cur, &P2);
      }
    }
    int top = 256;
    for (; top >= 0; --top) {
      uint64_t j = 0;
      while (j < npts && naf[257 * j + top] == 0) ++j;
      if (j < npts) break;
    }
    ge_p2 r;
    ge_p2_0(&r);
    ge_p1p1 t;
    ge_p3 u;
    for (int i = top; i >= 0; --i) {
      ge_dbl(&t, &r);
      for (uint64_t j = 0; j < npts; ++j) {
        const int d = naf[257 * j + i];
        if (!d) continue;
        p1p1_to_p3(&u, &t);
        ge_add_cached(&t, &u, &tab[8 * j + (d > 0 ? d : -d) / 2], d < 0);
      }
      p1p1_to_p2(&r, &t);
    }
    ok = fe_iszero(&r.X) && fe_eq(&r.Y, &r.Z);
  }
  free(pts);
  free(sc);
  free(tab);
  free(naf);
  return ok;
}

/* Certificate::verify over G certificates (primary/src/messages.rs:189-215),
 * signature and digest work only (the committee stake/quorum checks are a few
 * map lookups): header id == SHA-512(header preimage)[..32], header signature
 * verify_strict, certificate digest SHA-512(id || round || origin)[..32], and
 * dalek's verify_batch of the votes over it.  CPU BASELINE ONLY (bench.py
 * config 3).  out: one byte per certificate. */
typedef struct {
  const uint8_t *hdr, *ids, *hpk, *hsig, *cpre, *vpk, *vsig;
  const uint64_t *hoff, *hlen, *first;
  const uint32_t *cnt;
  uint64_t lo, hi;
  uint8_t *out;
} cjob;

static void *cert_worker(void *p) {
  cjob *j = (cjob *)p;
  uint8_t zkey[32] = {0};
  for (uint64_t g = j->lo; g < j->hi; ++g) {
    uint8_t h[64], d[64];
    ntor_sha512(j->hdr + j->hoff[g], j->hlen[g], h);
    int ok = memcmp(h, j->ids + 32 * g, 32) == 0;
    ok = ok && ntor_ed25519_verify_strict(j->hpk + 32 * g, j->hsig + 64 * g, j->ids + 32 * g, 32);
    if (ok) {
      ntor_sha512(j->cpre + 72 * g, 72, d);
      memcpy(zkey, &g, sizeof g);
      ok = ntor_ed25519_verify_batch_dalek(j->vpk + 32 * j->first[g], j->vsig + 64 * j->first[g], j->cnt[g], d, 32,
                                           zkey);
    }
    j->out[g] = (uint8_t)ok;
  }
  return NULL;
}

void ntor_certificates_verify_many(const uint8_t *hdr, const uint64_t *hoff, const uint64_t *hlen,
                                   const uint8_t *ids, const uint8_t *hpk, const uint8_t *hsig,
                                   const uint8_t *cpre, const uint8_t *vpk, const uint8_t *vsig,
                                   const uint64_t *first, const uint32_t *cnt, uint64_t G, uint8_t *out,
                                   int nthreads) {
  ensure_consts();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint64_t)nthreads > G) nthreads = G ? (int)G : 1;
  pthread_t th[256];
  cjob jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    cjob c = {hdr, ids, hpk, hsig, cpre, vpk, vsig, hoff, hlen, first, cnt, G * t / nthreads, G * (t + 1) / nthreads,
              out};
    jobs[t] = c;
    if (nthreads == 1) cert_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, cert_worker, &jobs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
