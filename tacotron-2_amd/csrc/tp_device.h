// Device helpers shared by the persistent training kernels (train_persist.hip forward,
// train_bwd_persist.hip backward): branch-free activations, bf16 packing, AGPR residency,
// buffer-resource loads / write-through stores of exchanged data, the bounded flag spins and
// the publish step of the chip-wide hand-offs.  Args: any argument struct with `unsigned* flags`
// ([phases][TP_NREP][TP_NB]) and `int* ctl` ([0] = 1 + phase of a failed wait).
#pragma once
#include "train_persist.h"

namespace tt2 {

typedef __bf16 tp_bf8 __attribute__((ext_vector_type(8)));
typedef unsigned tp_u2 __attribute__((ext_vector_type(2)));
typedef unsigned tp_u4 __attribute__((ext_vector_type(4)));
typedef float tp_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned tp_gu32;
typedef __attribute__((address_space(1))) int tp_gi32;
typedef __attribute__((address_space(1))) unsigned long long tp_gu64;
#define TP_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
constexpr long long TP_TIMEOUT = 200000000LL;  // 2 s of s_memrealtime (100 MHz)
// branch-free tanh (tanhf's two paths diverge per lane): odd Taylor polynomial below |x| = 1/16
// (truncation < 2e-13), (1 - e)·rcp(1 + e) with e = exp(-2|x|) above (the subtraction exact; v_rcp_f32
// instead of the IEEE division sequence __fdividef compiles to here: the result within ~1e-6 relative); the
// sign restored by copysign
__device__ __forceinline__ float tp_tanh(float x) {
  const float ax = fabsf(x), x2 = x * x;
  const float p = x * (1.f + x2 * (-1.f / 3.f + x2 * (2.f / 15.f + x2 * (-17.f / 315.f))));
  const float e = __expf(-2.f * ax);
  const float r = copysignf((1.f - e) * __builtin_amdgcn_rcpf(1.f + e), x);
  return ax < 0.0625f ? p : r;
}

// v_exp_f32 + v_rcp_f32 (relative error < 4e-7, no IEEE division on the per-step chain)
__device__ __forceinline__ float tp_sigm(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tp_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float tp_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ unsigned tp_pack(float lo, float hi) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)lo) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)hi) << 16);
}
// explicit AGPR residency for the per-row constants the attention reads once per step (keys, the
// values quarter): the VGPRs stay free for the LSTM products' fragments in flight
__device__ __forceinline__ float tp_aput(float v) {
  float r;
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ float tp_aget(float r) {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(r));
  return v;
}

// sc1 (L1-bypassing) loads and write-through stores of exchanged data; offsets in bytes
__device__ __forceinline__ auto tp_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// plain buffer store / load of one dword: per-lane byte offset + uniform byte offset (no per-lane
// 64-bit addresses in the step loop, where the compiler would keep one per store site alive)
__device__ __forceinline__ void tp_bst(const void* base, int vbyte, int sbyte, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), tp_rsrc(base), vbyte, sbyte, 0);
}
__device__ __forceinline__ void tp_st8(void* base, int byte_off, tp_u2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, tp_rsrc(base), byte_off, 0, 16);
}
__device__ __forceinline__ void tp_st16(void* base, int byte_off, tp_u4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, tp_rsrc(base), byte_off, 0, 16);
}

// Wave-uniform bounded spin until cond() holds on every lane; false on timeout or a peer's failure
// (ctl[0] != 0), the failing phase recorded there.
template <class Args, class F>
__device__ __forceinline__ bool tp_spin(const Args& a, int ph, F cond) {
  long long t0 = 0;
  for (unsigned spin = 0;; ++spin) {
    if (__all(cond())) return true;
    if ((spin & 63) == 0) {
      const long long now = __builtin_amdgcn_s_memrealtime();
      if (spin == 0) {
        t0 = now;
      } else if (__hip_atomic_load((tp_gi32*)a.ctl, TP_RLX) != 0 || now - t0 > TP_TIMEOUT) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store((tp_gi32*)a.ctl, 1 + ph, TP_RLX);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ unsigned tp_flag(const unsigned* f) {
  return __hip_atomic_load((tp_gu32*)const_cast<unsigned*>(f), TP_RLX);
}
// wave poll: flags of producers [base, base + n) of phase ph reached tag (this XCD group's replica)
template <class Args>
__device__ __forceinline__ bool tp_poll(const Args& a, int ph, int base, int n, unsigned tag) {
  const unsigned* f = a.flags + ((long)ph * TP_NREP + (blockIdx.x & (TP_NREP - 1))) * TP_NB + base;
  const int lane = threadIdx.x & 63;
  return tp_spin(a, ph, [&] { return lane >= n || tp_flag(f + lane) >= tag; });
}
// every wave drains its stores, one barrier, then this work-group's flag in every replica
template <class Args>
__device__ __forceinline__ void tp_publish(const Args& a, int ph, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < TP_NREP)
    __hip_atomic_store((tp_gu32*)(a.flags + ((long)ph * TP_NREP + threadIdx.x) * TP_NB + blockIdx.x), tag, TP_RLX);
}

// 16-byte buffer load issued by inline asm: the compiler schedules at most two of its own loads
// ahead of their MFMAs here (measured: one round trip per fragment), so a batch of fragments is
// issued back to back and waited for once (tp_wait), one L2 round trip per batch.  The compiler's
// hazard recognizer does not see into the asm: an soffset / resource SGPR it has just reloaded
// from a spill lane (v_readlane, a VALU write of an SGPR) needs 5 wait states before a VMEM
// instruction reads it, hence the s_nop 4 in front of every load (without it the load reads the
// stale SGPR: a wrong offset, measured as a device fault)
template <bool SC1>
__device__ __forceinline__ tp_bf8 tp_ldx4(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
  tp_bf8 r;
  if constexpr (SC1)
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen sc1" : "=v"(r) : "v"(vo), "s"(rs), "s"(so) : "memory");
  else
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(vo), "s"(rs), "s"(so) : "memory");
  return r;
}
// wait for every load of the batch; the fragments pass through as operands so no use is scheduled
// above the wait
template <int N>
__device__ __forceinline__ void tp_wait(tp_bf8 (&f)[N]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

}  // namespace tt2
