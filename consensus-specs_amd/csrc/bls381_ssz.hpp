// SSZ hash_tree_root / signing_root of fixed-size containers on gfx950: the
// message_hash producer in front of bls_verify.
//
// Reference: test_libs/pyspec/eth2spec/utils/ssz/ssz_impl.py:143-163
// (hash_tree_root, signing_root), :110-123 (pack, chunkify), and
// utils/merkle_minimal.py merkleize_chunks (zero-chunk padding to a power of
// two, a single chunk is its own root).  A fixed-size SSZ value serializes to
// the concatenation of its fields, so a root is a small program over the
// item's serialized bytes; bls381_amd/ssz.py compiles a type into it:
//   SSZ_CHUNK off len : push bytes [off, off+len) zero-padded to 32 (len <= 32)
//   SSZ_MERKLE k      : pop k chunks, pad with zero chunks to a power of two,
//                       merkleize, push the root
// One lane runs the program for one item; the chunk stack lives in scratch.
#pragma once
#include "bls381_hash.hpp"

namespace bls381 {

enum : uint32_t { SSZ_CHUNK = 1, SSZ_MERKLE = 2 };
constexpr int SSZ_STACK = 64;    // chunks
constexpr int SSZ_PROG_MAX = 512;  // u32 words

// SHA-256 of two 32-byte chunks (one data block + the constant padding block)
BLS_DEV_INLINE void sha256_pair(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t blk[16];
  for (int i = 0; i < 8; ++i) { blk[i] = l[i]; blk[8 + i] = r[i]; }
  sha256_compress(h, blk);
  for (int i = 0; i < 16; ++i) blk[i] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512;                 // bit length of the 64-byte message
  sha256_compress(h, blk);
  for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// Runs `prog` over one serialized item; the root (8 big-endian words) is left in
// root.  Returns false on a malformed program (stack over/underflow).
BLS_DEV_INLINE bool ssz_run(uint32_t root[8], const uint8_t* item, const uint32_t* prog, uint32_t plen,
                           uint32_t (*stk)[8]) {
  int sp = 0;
  for (uint32_t pc = 0; pc < plen;) {
    const uint32_t op = prog[pc];
    if (op == SSZ_CHUNK && pc + 2 < plen) {
      const uint32_t off = prog[pc + 1], len = prog[pc + 2];
      pc += 3;
      if (sp >= SSZ_STACK || len > 32) return false;
      for (int w = 0; w < 8; ++w) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b) {
          const uint32_t k = 4 * w + b;
          v = (v << 8) | (k < len ? item[off + k] : 0u);
        }
        stk[sp][w] = v;
      }
      ++sp;
    } else if (op == SSZ_MERKLE && pc + 1 < plen) {
      const uint32_t k = prog[pc + 1];
      pc += 2;
      if (k == 0 || (int)k > sp) return false;
      uint32_t p = 1;
      while (p < k) p <<= 1;
      const int base = sp - (int)k;
      if (base + (int)p > SSZ_STACK) return false;
      for (uint32_t j = k; j < p; ++j)
        for (int w = 0; w < 8; ++w) stk[base + j][w] = 0;
      for (uint32_t width = p; width > 1; width >>= 1)
        for (uint32_t j = 0; j < width / 2; ++j) sha256_pair(stk[base + j], stk[base + 2 * j], stk[base + 2 * j + 1]);
      sp = base + 1;
    } else {
      return false;
    }
  }
  if (sp != 1) return false;
  for (int w = 0; w < 8; ++w) root[w] = stk[0][w];
  return true;
}

}  // namespace bls381
