// Basic types and qualifiers shared by the gfx950 kernels and the host unit-test
// build of the same arithmetic (DESIGN.md "One source, two compilers").
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
// keep the scheduler from interleaving independent phases (bounds live ranges)
#if defined(__HIP_DEVICE_COMPILE__)
#define BLS_PHASE() __builtin_amdgcn_sched_barrier(0)
// true on every active lane when c holds on any of them (a wave-uniform branch)
#define BLS_ANY(c) (__builtin_amdgcn_ballot_w64((c)) != 0)
#else
#define BLS_PHASE() ((void)0)
#define BLS_ANY(c) (c)
#endif
#define BLS_HD __host__ __device__
#define BLS_INLINE __host__ __device__ __forceinline__
#define BLS_NOINLINE __host__ __device__ __attribute__((noinline))
// always inlined on the device (a non-inlined function taking references or
// pointers into its caller's private memory makes flat accesses to the private aperture);
// an ordinary inline function in the host unit-test build, which keeps g++ fast
#define BLS_DEV_INLINE __host__ __device__ __forceinline__
#define BLS_CONST __device__ __constant__ static constexpr
#else
#define BLS_PHASE() ((void)0)
#define BLS_ANY(c) (c)
#define BLS_HD
#define BLS_INLINE inline __attribute__((always_inline))
#define BLS_NOINLINE __attribute__((noinline))
#define BLS_DEV_INLINE inline
#define BLS_CONST static constexpr
#endif

namespace bls381 {

// Fp element: 14 limbs of 28 bits held in u32 words, little-endian, Montgomery
// form with R = 2^392.  Stored values keep every limb < 2^28 and value < 2q
// (DESIGN.md "Fp representation"); Fp multiplication accumulates each 28x28-bit
// partial product in place into a 64-bit column (one v_mad_u64_u32 per product).
constexpr int FP_LIMBS = 14;
constexpr int FP_BITS = 28;
constexpr uint32_t FP_MASK = (1u << 28) - 1;
struct fp_t { uint32_t w[14]; };
// Fp2 = Fp[u]/(u^2+1): c0 + c1 u
struct fp2_t { fp_t c0, c1; };
// Fp6 = Fp2[v]/(v^3 - (1+u)) and Fp12 = Fp6[w]/(w^2 - v): c0 + c1 w, generic
// over the Fp2 representation E (fp2_t here; the lane-pair fp2p_t of
// bls381_pair.hpp in the kernels)
template <class E> struct fp6_g { E c0, c1, c2; };
template <class E> struct fp12_g { fp6_g<E> c0, c1; };
using fp6_t = fp6_g<fp2_t>;
using fp12_t = fp12_g<fp2_t>;
// Fp2 held by an adjacent lane pair: lane 2i+p holds coefficient p of item i
struct fp2p_t { fp_t v; };

// Jacobian points (X/Z^2, Y/Z^3); Z == 0 is the point at infinity
struct g1_jac { fp_t x, y, z; };
struct g2_jac { fp2_t x, y, z; };
struct g1_aff { fp_t x, y; };
struct g2_aff { fp2_t x, y; };

}  // namespace bls381
