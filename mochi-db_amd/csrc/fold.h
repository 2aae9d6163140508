// fold.h — the per-key fold matrix of k_rsa_pow (rsa_pow.hip).
//
// One squaring of x < 2^2064 (74 limbs of 28 bits) is
//   t = x^2                                        (148 limbs, VALU)
//   x' = t_lo + sum_{j<75, b<4} byte_b(t_{73+j}) * R_{j,b},   R_{j,b} = 2^(28(73+j)+8b) mod n
// with t_lo = limbs 0..72.  The sum is an int8 GEMM on the matrix cores: the
// key's R_{j,b} written as balanced mixed-radix digits (three signed bytes and
// a signed nibble per 28-bit limb: 74 x 4 = 296 output rows) times the 300
// bytes of t_hi, biased to signed by -128.  fold < 75 * (3*255 + 15) * n
// < 2^15.84 * 2^2048, so x' < 2^2064 again and the chain never overflows.
//
// Image layout = the MFMA A-operand fragments of v_mfma_i32_32x32x32_i8 in
// issue order: [M-tile 10][K-step 10][lane 64][16 bytes], lane l holding row
// 32*mt + (l & 31) (output limb 8mt + (l&31)/4, digit slot (l&31)%4) and the
// K slots of half h = l >> 5: t_hi limb 8*ks + 4h + i, byte b at byte 4i + b.
#pragma once
#include <stdint.h>

namespace mochi {

constexpr int kFoldF = 73;    // fold point: t_lo = limbs [0, 73)
constexpr int kFoldNH = 75;   // t_hi = limbs 73..147
constexpr int kFoldKS = 10;   // K-steps (8 t_hi limbs = 32 bytes each)
constexpr int kFoldMT = 10;   // M-tiles (8 output limbs each)
constexpr int kFoldImgBytes = kFoldMT * kFoldKS * 64 * 16;  // 102,400 B (one CU's LDS holds one key)
constexpr int kFoldLimbs = 74;
constexpr uint32_t kBucketAlign = 512;  // k_rsa_pow block = 8 waves of one signer
// The fold's signed B operand: every t_hi limb is an int32 whose bytes 0..2 are
// biased to signed (XOR 0x80: byte - 128) and whose byte 3 is taken as a signed
// digit as it is, so a limb may be negative (kara_dev.h leaves t[37..111]
// signed).  cadd adds the bias back (128 * sum_{j, b<3} R_{j,b}) plus
// kFoldOffN * n, which keeps x' positive: every top digit is >= -32 (|t_j| <
// 2^29) and t_lo > -n.  Then 0 < x' < 2^2064 (tests/fold_model.py).
constexpr uint32_t kFoldBias = 0x00808080u;
constexpr int kFoldOffN = 2401;

struct FoldKey {
  int8_t img[kFoldImgBytes];
  // the -128 bias of t_hi bytes 0..2 removes 128 * R_{j,b} per such K slot:
  // cadd = 128 * sum_{j, b<3} R_{j,b} + kFoldOffN * n (< 2^2064), added back
  // once as 74 normalised limbs
  uint32_t cadd[kFoldLimbs];
  // k_rsa_final's constant: cadd + n - Cpad (Cpad = the EMSA-PKCS1-v1_5
  // encoding with a zero digest), so its fold yields x + n - EM + H directly
  uint32_t cnc[kFoldLimbs];
  uint8_t pad[1024 - 2 * kFoldLimbs * 4];
};
static_assert(sizeof(FoldKey) == kFoldImgBytes + 1024, "FoldKey layout");

}  // namespace mochi
