// Persistent Tacotron-2 decoder for MI355X (gfx950): the whole dynamic_decode loop
// (tacotron.py:349-354 over TacotronDecoderCell.__call__, Architecture_wrappers.py:197-267) as ONE
// launch of 256 work-groups, one per CU.
//
// Why: at batch 32 the decoder step is a chain of small dependent GEMVs.  Streaming the 73 MB of
// step weights from HBM every step bounds a per-launch design at ~13 us/step plus ~1.5 us per
// kernel boundary.  The chip holds 256 x (512 KB VGPR + 160 KB LDS): every step weight fits
// on-chip, so each work-group keeps its LSTM column tile resident (input rows in registers,
// recurrent rows in LDS) and the per-step HBM traffic drops to the activations exchanged between
// work-groups.
//
// Roles of work-group g (every work-group has all three):
//   LSTM   hidden units pd_unit(g, 0..3) of both layers = one 16-column gate tile (pd_lstm_cols
//          order): one AF float4 per row, so the h1/h2 exchange stores are whole 16-byte stores
//   row    attention row b = (g&7)*4 + ((g>>3)&3), slice j = g>>5: attention dims [16j, 16j+16),
//          context channels [64j, 64j+64), prenet-L2 outputs [32j, 32j+32).  The 8 siblings of a
//          row have equal g%8 (one XCD under round-robin placement: faster, never required).
//   proj   g < 176: frame/stop/prenet-L1 projection tile g%22, K split g/22
//
// One step t (tag = t+1, buffers by parity t&1).  "wait X" = poll the producers' X flags; every
// payload byte is stored write-through (sc1) and drained before the flag, every read of it is an
// sc1 load (MI355X_MICROARCH.md § visibility, Valid forms row 1).
//   A  wait PRE(all)  [stop rule of t-1 from the flags' low bits]  L1 gates += prenet rows
//      (context, style and recurrent terms were accumulated earlier) -> h1_new -> H1, flag H1
//      tail: RG2 = (1-z)·h2_new(t-1)·W2h + z·RG2      (zoned-state recurrence, linear)
//   B  wait H1(all)   L2 gates = h1_new·W2i + RG2 -> h2_new -> H2, flag H2
//      tail: RG1 = (1-z)·h1_new(t)·W1h + z·RG1
//   C  wait H2(all)   q_j = h2_new[b]·Wq[:, j-slice]; partial energies over all encoder steps -> E
//      tail (proj blocks): projection partial += h2 rows of its K split
//   D  wait E(row)    Σ_j energies, masks, softmax, cum/max_att, context slice -> CTX, flag CTX
//      tail: location features of step t+1 (cum is local to the row's siblings)
//   E  proj blocks: wait CTX(slice) -> projection partial += context rows -> PP, flag PP
//   F  wait PP(all)   frame/stop (row), stop bit, prenet of step t+1 -> PRE, flag PRE|stop
//      tail: wait CTX(all): L1 context rows for step t+1; Σ_{t<len} align of every row
// Spins are bounded (2 s): a timeout or a peer's error makes every work-group exit and the host
// reports TT2_ERR_HIP.
#include "decode_persist.h"

namespace tt2 {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(1))) float pd_gf32;
typedef __attribute__((address_space(1))) unsigned pd_gu32;
typedef __attribute__((address_space(1))) int pd_gi32;
typedef __attribute__((address_space(1))) unsigned long long pd_gu64;
#define PD_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// h1 hand-off protocol (A/B switch): 0 = write-through stores, drain, replicated flag, consumer
// polls its 32 producers' flags then loads; 1 = self-tagged values, flag as a hint polled after an
// optimistic load missed; 2 = self-tagged values, the consumer re-loads the data until it is valid
#ifndef PD_TAG_H1
#define PD_TAG_H1 0
#endif
constexpr long long PD_TIMEOUT = 200000000LL;  // 2 s of s_memrealtime (100 MHz)
constexpr int PD_LDS_FLOATS = 16384 * 2 + 4096 + 512 * 5 + 288 + 256 * 2 + 32 + 16 + 16 + 16 + 512;  // 159.6 KB

// write-through (sc1) stores and L1-bypassing (sc1) loads of hand-off data
__device__ __forceinline__ float pd_ld(const float* p) {
  return __hip_atomic_load((pd_gf32*)const_cast<float*>(p), PD_RLX);
}
__device__ __forceinline__ void pd_st(float* p, float v) { __hip_atomic_store((pd_gf32*)p, v, PD_RLX); }
__device__ __forceinline__ f32x4 pd_ld4(const float* base, int i4) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, i4 * 16, 0, 16));
}

// Wave-uniform bounded spin: poll until cond() holds on every lane.  false on timeout (2 s) or
// when a peer reported a failure in ctl[2]; the failing phase is recorded there.
template <class F>
__device__ __forceinline__ bool pd_spin(const PdArgs& a, int ph, int lane, F cond) {
  long long t0 = 0;
  for (unsigned spin = 0;; ++spin) {
    if (__all(cond())) return true;
    if ((spin & 63) == 0) {
      const long long now = __builtin_amdgcn_s_memrealtime();
      if (spin == 0) {
        t0 = now;
      } else if (__hip_atomic_load((pd_gi32*)(a.ctl + 2), PD_RLX) != 0 || now - t0 > PD_TIMEOUT) {
        if (lane == 0) __hip_atomic_store((pd_gi32*)(a.ctl + 2), 1 + ph, PD_RLX);
        return false;
      }
    }
    for (int z = 0; z < a.poll_sleep; ++z) __builtin_amdgcn_s_sleep(1);  // back off: pollers load the memory system
  }
}

__device__ __forceinline__ unsigned pd_flag(const unsigned* f) {
  return __hip_atomic_load((pd_gu32*)const_cast<unsigned*>(f), PD_RLX);
}

// Wave-level poll: every flag f[base + i*stride] (i < n <= 64) of phase ph has (v >> shift) >= need.
__device__ __forceinline__ bool pd_poll(const PdArgs& a, int ph, int base, int stride, int n, unsigned need, int shift,
                                        int lane) {
  const unsigned* f = a.flags + ph * PD_NB + base;
  return pd_spin(a, ph, lane, [&] { return lane >= n || (pd_flag(f + lane * stride) >> shift) >= need; });
}

// Wave-level poll for ALL producers g < nprod of phase ph, two-level so that no flag line has more
// than 32 pollers (256 pollers on one line serialise at its memory channel, ~3 us per hop): the
// consumers form groups of 8 (x = g/8, member s = g%8); member s waits for producers
// [32s, 32s+32) (one 128-B line) and raises flags2[ph][x][s], then waits for its group's 8 flags.
__device__ __forceinline__ bool pd_poll_all(const PdArgs& a, int ph, int nprod, unsigned need, int shift, int lane,
                                            bool sweep_first) {
  const int g = blockIdx.x, x = g >> 3, s = g & 7;
  const unsigned* f = a.flags + ph * PD_NB + 32 * s;
  unsigned* f2 = a.flags2 + ph * PD_NB + 8 * x;
  if (sweep_first) {  // one sweep of all producers first: one round trip when the hand-off already
                      // landed (waits behind a long tail); not where all 256 arrive at once
    const unsigned* fa = a.flags + ph * PD_NB;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pidx = lane + 64 * i;
      ok = ok && (pidx >= nprod || (pd_flag(fa + pidx) >> shift) >= need);
    }
    if (__all(ok)) {
      if (lane == 0) __hip_atomic_store((pd_gu32*)(f2 + s), need, PD_RLX);  // members may be polling it
      return true;
    }
  }
  if (!pd_spin(a, ph, lane, [&] { return lane >= 32 || 32 * s + lane >= nprod || (pd_flag(f + lane) >> shift) >= need; }))
    return false;
  if (lane == 0) __hip_atomic_store((pd_gu32*)(f2 + s), need, PD_RLX);
  return pd_spin(a, ph, lane, [&] { return lane >= 8 || pd_flag(f2 + lane) >= need; });
}

// Wave-level poll of the 32 producers [base, base+32) of h-phase r (0: H1, 1: H2) on this work-group's
// replica of their flag line (replica g%8: 32 pollers per line).  Each wave waits only for the
// producers of the rows it loads, so early waves start their MFMAs while late producers finish.
__device__ __forceinline__ bool pd_poll_rep(const PdArgs& a, int ph, int r, int base, unsigned need, int lane,
                                            int n = 32) {
  const unsigned* f = a.rflags + (r * PD_NREP + (blockIdx.x & (PD_NREP - 1))) * PD_NB + base;
  return pd_spin(a, ph, lane, [&] { return lane >= n || pd_flag(f + lane) >= need; });
}

// Block-level waits: wave 0 polls, the work-group joins at a barrier (result via LDS slot).
template <class F>
__device__ __forceinline__ bool pd_block_wait(int* slot, F poll) {
  if (threadIdx.x < 64) {
    const bool ok = poll();
    if (threadIdx.x == 0) *slot = ok;
  }
  __syncthreads();
  return *slot != 0;
}

// Data-tagged 8-byte granule {tag, fp32 bits}: the data is the flag (Guideline 16 R2) -- no drain,
// no separate flag round trip.  For the small intra-row exchanges (energies, projection partials).
__device__ __forceinline__ void pd_put(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store((pd_gu64*)g, ((unsigned long long)tag << 32) | __float_as_uint(v), PD_RLX);
}
// Each active lane fetches N granules base[off + i*stride] (base wave-uniform) until every tag ==
// tag (wave-uniform bounded spin).  false: timeout or a peer failed.
template <int N>
__device__ __forceinline__ bool pd_take(const PdArgs& a, int ph, const unsigned long long* base, int off, int stride,
                                        unsigned tag, bool active, float (&v)[N]) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned long long*>(base), (short)0, 0x7fffffff, 0x00020000);
  long long t0 = 0;
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
    if (active) {  // every load issued before any tag is compared (no short-circuit: a branch per
                   // granule would let the compiler serialise the loads)
      unsigned tags[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off * 8, i * stride * 8, 16);  // sc1
        v[i] = __uint_as_float(x[0]);
        tags[i] = x[1];
      }
      unsigned bad = 0u;
#pragma unroll
      for (int i = 0; i < N; ++i) bad |= tags[i] ^ tag;
      ok = bad == 0u;
    }
    if (__all(ok)) return true;
    if ((spin & 31) == 0) {
      const long long now = __builtin_amdgcn_s_memrealtime();
      if (spin == 0) {
        t0 = now;
      } else if (__hip_atomic_load((pd_gi32*)(a.ctl + 2), PD_RLX) != 0 || now - t0 > PD_TIMEOUT) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store((pd_gi32*)(a.ctl + 2), 1 + ph, PD_RLX);
        return false;
      }
    }
    for (int z = 0; z < a.poll_sleep; ++z) __builtin_amdgcn_s_sleep(1);
  }
}

// Self-tagged exchange values (h1, h2, context slices, Σ align): bit 0 of every fp32 value written at
// step t carries tb(t) = ((t >> 1) & 1) ^ 1.  A buffer of parity t & 1 otherwise holds step t-2's
// values (the other tag bit) or the per-launch zeros (bit 0 = 0 never matches steps 0, 1), so a
// consumer can check every value it loaded: the producer needs no drain before its flag, and the
// consumer no flag round trip before its data load when the data has landed.  The flag stays as a
// hint polled only after an optimistic load missed.  Cost: one ulp (2^-23 relative) on exchanged
// values, below the split fp16x3 products' own 2^-22.
__device__ __forceinline__ unsigned pd_tb(int t) { return ((unsigned)(t >> 1) & 1u) ^ 1u; }
__device__ __forceinline__ float pd_tag(float v, unsigned tb) { return __uint_as_float((__float_as_uint(v) & ~1u) | tb); }
__device__ __forceinline__ bool pd_ok1(float v, unsigned tb) { return ((__float_as_uint(v) ^ tb) & 1u) == 0u; }
__device__ __forceinline__ bool pd_ok4(const f32x4& v, unsigned tb) {
  return (((__float_as_uint(v[0]) ^ tb) | (__float_as_uint(v[1]) ^ tb) | (__float_as_uint(v[2]) ^ tb) |
           (__float_as_uint(v[3]) ^ tb)) & 1u) == 0u;
}

// Wave-level take of N self-tagged values X[idx(i)] (sc1 loads; V = f32x4 or float).  The first pass
// is optimistic; after a miss hint() runs once (a flag poll: the producers have at least issued
// their stores) and the loads repeat until every value carries tb (bounded spin; one copy of the
// loads in the loop keeps the register footprint of the fast path).  false: timeout or a peer failed.
__device__ __forceinline__ f32x4 pd_ldv(const float* X, int i, f32x4) { return pd_ld4(X, i); }
__device__ __forceinline__ float pd_ldv(const float* X, int i, float) { return pd_ld(X + i); }
__device__ __forceinline__ bool pd_okv(const f32x4& v, unsigned tb) { return pd_ok4(v, tb); }
__device__ __forceinline__ bool pd_okv(float v, unsigned tb) { return pd_ok1(v, tb); }
template <int N, class V, class I, class H>
__device__ __forceinline__ bool pd_takev(const PdArgs& a, int ph, const float* X, I idx, unsigned tb, V (&v)[N],
                                         H hint) {
  long long t0 = 0;
  for (unsigned spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = pd_ldv(X, idx(i), v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) ok = ok && pd_okv(v[i], tb);
    if (__all(ok)) return true;
    if (spin == 0) {
      if (!hint()) return false;
      t0 = __builtin_amdgcn_s_memrealtime();
      continue;
    }
    if ((spin & 31) == 0) {
      if (__hip_atomic_load((pd_gi32*)(a.ctl + 2), PD_RLX) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > PD_TIMEOUT) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store((pd_gi32*)(a.ctl + 2), 1 + ph, PD_RLX);
        return false;
      }
    }
    for (int z = 0; z < a.poll_sleep; ++z) __builtin_amdgcn_s_sleep(1);
  }
}
template <int N, class I, class H>
__device__ __forceinline__ bool pd_take4(const PdArgs& a, int ph, const float* X, I idx, unsigned tb, f32x4 (&v)[N],
                                         H hint) {
  return pd_takev<N>(a, ph, X, idx, tb, v, hint);
}
template <int N, class I, class H>
__device__ __forceinline__ bool pd_take1(const PdArgs& a, int ph, const float* X, I idx, unsigned tb, float (&v)[N],
                                         H hint) {
  return pd_takev<N>(a, ph, X, idx, tb, v, hint);
}

// LSTM epilogue store: the 4 hidden units this work-group owns for row em (pd_unit) are one AF
// float4, held by the 4 consecutive lanes eu = 0..3; lane eu = 0 writes it as ONE 16-byte
// write-through store (rows 0..15 / 16..31 of a work-group fill 256 contiguous bytes each),
// every value self-tagged with tb (tb = ~0u: stored as computed, for the flag protocol).
__device__ __forceinline__ void pd_st_h4(float* X, int em, int u0, float hn, int lane, unsigned tb) {
  const int src = lane & ~3;
  const auto tg = [&](float v) { return tb > 1u ? v : pd_tag(v, tb); };
  const float v0 = tg(__shfl(hn, src)), v1 = tg(__shfl(hn, src + 1));
  const float v2 = tg(__shfl(hn, src + 2)), v3 = tg(__shfl(hn, src + 3));
  if ((lane & 3) == 0) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(X, (short)0, 0x7fffffff, 0x00020000);
    const u32x4 d = {__float_as_uint(v0), __float_as_uint(v1), __float_as_uint(v2), __float_as_uint(v3)};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, af_idx(em, u0) * 4, 0, 16);  // sc1
  }
}

// Every storing wave drains its sc1 stores, then one lane raises this work-group's flag.
__device__ __forceinline__ void pd_publish(const PdArgs& a, int ph, unsigned val, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store((pd_gu32*)(a.flags + ph * PD_NB + blockIdx.x), val, PD_RLX);
}

// Flag hint of self-tagged data: no drain (the consumers check the tags), the barrier only so the
// flag follows every wave's stores in issue order.
__device__ __forceinline__ void pd_hint(const PdArgs& a, int ph, unsigned val, int tid) {
  __syncthreads();
  if (tid == 0) __hip_atomic_store((pd_gu32*)(a.flags + ph * PD_NB + blockIdx.x), val, PD_RLX);
}
__device__ __forceinline__ void pd_hint_rep(const PdArgs& a, int r, unsigned val, int tid) {
  __syncthreads();
  if (tid < PD_NREP) __hip_atomic_store((pd_gu32*)(a.rflags + (r * PD_NREP + tid) * PD_NB + blockIdx.x), val, PD_RLX);
}

// pd_publish to every replica of h-phase r's flag line.
__device__ __forceinline__ void pd_publish_rep(const PdArgs& a, int r, unsigned val, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < PD_NREP) __hip_atomic_store((pd_gu32*)(a.rflags + (r * PD_NREP + tid) * PD_NB + blockIdx.x), val, PD_RLX);
}

// acc(rows 0..15 | 16..31) += A(k-group) · W(k-group, 16 columns), split fp16x3 (common.h)
__device__ __forceinline__ void kg_mfma(const f32x4& a0, const f32x4& a1, const f32x4& bw, f32x4& c0, f32x4& c1) {
  kg_mfma_x3(a0, a1, bw, c0, c1);
}

// Partial tile of wave w -> red[w][32][16] (the MFMA D layout transposed to row-major).
__device__ __forceinline__ void put_partials(const f32x4& acc0, const f32x4& acc1, float* red, int w, int lane) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = lane & 15, m = (lane >> 4) * 4 + r;
    red[w * 512 + m * 16 + n] = acc0[r];
    red[w * 512 + (m + 16) * 16 + n] = acc1[r];
  }
}
template <int NW>
__device__ __forceinline__ float sum_partials(const float* red, int idx) {
  float v = red[idx];
#pragma unroll
  for (int ww = 1; ww < NW; ++ww) v += red[ww * 512 + idx];
  return v;
}

// Barrier of the 4 tail waves (4..7) through an LDS counter: the chain waves never take part, so
// a tail job can finish its reduction while wave 0 is still polling.
__device__ __forceinline__ void tail_bar(int* ctr, unsigned& gen, int lane) {
  gen += 4;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while ((unsigned)__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
    __builtin_amdgcn_s_sleep(0);
}

#define PD_STAMP(i)                                                                   \
  do {                                                                                \
    if (stp && tid == 0) stp[g * 32 + (i)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)

// TM: encoder steps covered (256, or 512 for T_in > 256).  TM = 512 keeps the values of positions
// [0, 256) resident like TM = 256 and streams those of [256, 512) from L2 / MALL every step (issued
// ahead of the energy take); its alignments live in the stage scratch (red + 2048: free during the
// softmax / context stage) so the cumulative alignments can take their place (15 + 512 + 17 floats).
// FL (diagnostic, TT2_PD_FLOOR=1): the "floor" instance -- every exchange, poll, barrier and load of the
// production kernel, with the arithmetic of the stage bodies removed (the MFMA products, the query /
// prenet / context dot products and the energies' tanh reductions consume their operands through an
// empty asm sink instead): the step time that is hand-offs + memory round trips alone.  Results garbage.
template <bool EMT, int TM, bool FL>
__global__ __launch_bounds__(PD_NT) void k_decode_persist(PdArgs a) {
  static_assert(TM == PD_TMAX || (TM == PD_TMAX_LONG && !EMT), "k_decode_persist geometry");
  static_assert(!FL || (!EMT && TM == PD_TMAX), "floor instance: the Tacotron decoder only");
  // split fp16x3 product, or (FL) its operands sunk
  const auto mm = [](const f32x4& a0, const f32x4& a1, const f32x4& bw, f32x4& c0, f32x4& c1) {
    if constexpr (FL) asm volatile("" ::"v"(a0), "v"(a1), "v"(bw));
    else kg_mfma(a0, a1, bw, c0, c1);
  };
  constexpr int NI = TM / 128;          // 16-position key / location tiles per wave
  constexpr int NWE = TM / 64;          // waves holding one energy per lane in the softmax
  constexpr int CWN = TM == PD_TMAX ? 288 : 544;  // cumulative-alignment floats (zero padded)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const sW1h = sm;              // [64 kg][64 lanes] f32x4: W1 recurrent rows of this tile
  float* const sW2h = sm + 16384;      // same for W2
  float* const red = sm + 32768;       // [8][512] partial tiles / stage scratch (tail jobs: during waits)
  float* const G = red + 4096;         // [32][16] spare tile
  float* const RG1 = G + 512;          // [32][16] zoned-h1 recurrent gate terms of the next L1
  float* const RG2 = RG1 + 512;        // same for L2
  float* const RGc = RG2 + 512;        // [32][16] context rows of the next L1
  float* const PPh = RGc + 512;        // [32][16] projection partial, h2 rows (proj blocks)
  float* const cw = PPh + 512;         // [15 + T + 16] cumulative alignments, zero padded (location conv)
  float* const al = TM == PD_TMAX ? cw + 288 : red + 2048;  // [TM] alignments of the step
  float* const x1 = cw + 544;          // [256] prenet layer-1 output of the row
  float* const ssa = x1 + 256;         // [32] Σ_{t<len} align of every row (last step)
  float* const qv = ssa + 32;          // [16] query slice
  float* const sc = qv + 16;           // softmax max / sum, Σ_{t<len} align of this row
  int* const si = reinterpret_cast<int*>(sc + 16);  // [0] max_att [1] done [2] wait result [3] tail ok [4] tail ctr
  const int g = blockIdx.x, tid_ = threadIdx.x;
  const int b = (g & 7) * 4 + ((g >> 3) & 3), j = g >> 5;
  const bool rowv = b < a.B;
  // EMT: 8 more projection tiles = the emotion query (pn >= PD_NTILE, "q" blocks, which also run the
  // attn_emt dense: output tile pn - PD_NTILE, K split pks); g >= PD_EG0: emotion rows 2(g-PD_EG0), +1
  constexpr int NTL = EMT ? PD_NTILE + PD_ENT : PD_NTILE;
  const bool isproj = g < NTL * PD_KSP;
  const int pn = g % NTL, pks = g / NTL;
  const bool isq = EMT && isproj && pn >= PD_NTILE;
  const int K1S = EMT ? a.K1 : PD_P + PD_E2;  // LSTM-1 critical rows per tile
  const int T = a.T_in;
  const int sib0 = (b >> 2) + 8 * (b & 3);  // siblings of row b: sib0 + 32*jj
  long long* const stp0 = a.stamps;

  // ---------------- prologue: resident weights and per-row constants ----------------
  const int tid = tid_, lane = tid & 63, w = tid >> 6;
  const int em = (tid >> 2) & 31, eu = tid & 3;  // LSTM epilogue thread (tid < 128) -> row, unit
  // every WF weight below comes pre-scaled by KG_SB (split fp16x3 range, common.h); the gate and
  // projection sums are unscaled by KG_UNSCALE where they are consumed
  f32x4 w1p[2], w2i[8];                          // chain: L1 prenet rows, L2 input rows (8 waves)
  {
    const f32x4* L1 = reinterpret_cast<const f32x4*>(a.l1_w + (long)g * K1S * 16);
    const f32x4* L2 = reinterpret_cast<const f32x4*>(a.l2_w + (long)g * PD_H * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i) w1p[i] = L1[(2 * w + i) * 64 + lane];  // pre-scaled (common.h)
#pragma unroll
    for (int i = 0; i < 8; ++i) w2i[i] = L2[(8 * w + i) * 64 + lane];
    const f32x4* L1h = reinterpret_cast<const f32x4*>(a.l1_wh + (long)g * PD_H * 16);
    const f32x4* L2h = reinterpret_cast<const f32x4*>(a.l2_wh + (long)g * PD_H * 16);
    f32x4* d1 = reinterpret_cast<f32x4*>(sW1h);
    f32x4* d2 = reinterpret_cast<f32x4*>(sW2h);
    for (int e = tid; e < PD_H * 4; e += PD_NT) {
      d1[e] = L1h[e];
      d2[e] = L2h[e];
    }
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 wpc = zero4;
  if (isproj && w < 4 && !isq) {
    const f32x4* PW = reinterpret_cast<const f32x4*>(a.proj_w + (long)pn * (PD_H + PD_E2) * 16);
    wpc = PW[(PD_H / 16 + 4 * pks + w) * 64 + lane];
  }
  // projection h2 rows of this split, k-group 8 pks + w (read in the C tail; L2-resident)
  const f32x4* const WPH = reinterpret_cast<const f32x4*>(a.proj_w + (long)pn * (PD_H + PD_E2) * 16) + (8 * pks) * 64;
  f32x4 w1c[4];  // L1 context rows, k-groups 16 + 4w + i of the tile
  {
    const f32x4* W1C = reinterpret_cast<const f32x4*>(a.l1_w + (long)g * K1S * 16) + (PD_P / 16 + 4 * w) * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) w1c[i] = W1C[i * 64 + lane];
  }
  f32x4 w1e = zero4, wdf = zero4;  // EMT: L1 emotion-block rows (k-group 48 + w); dense fragment (q blocks)
  if constexpr (EMT) {
    if (w < a.e_XW / 16)  // the block's k-groups ('style_tokens': 4 of the 8 waves)
      w1e = reinterpret_cast<const f32x4*>(a.l1_w + (long)g * K1S * 16)[((PD_P + PD_E2) / 16 + w) * 64 + lane];
    if (a.e_dense && isq && w < a.e_KC / 128)
      wdf = reinterpret_cast<const f32x4*>(a.e_wd + (long)(pn - PD_NTILE) * a.e_KC * 16)[(pks * (a.e_KC / 128) + w) * 64 + lane];
  }
  // location-conv WF fragments of this slice in LDS (2 KB after si: the same for every wave)
  f32x4* const swl = reinterpret_cast<f32x4*>(si + 16);
  if (tid < 128) swl[tid] = reinterpret_cast<const f32x4*>(a.loc_cw + (long)j * PD_KLP * 16)[tid];
  // LSTM epilogue constants of thread tid < 128 (row em, unit eu) in LDS, not VGPRs (the kernel
  // is at its 256-VGPR budget): cst[(k*4 + q)*128 + tid], k = 0 b1, 1 b2, 2 style term
  float* const cst = RG1;  // RG1 | RG2 | RGc: 1536 floats, otherwise unused
  const int u0 = pd_unit(g, 0);  // this work-group's hidden units pd_unit(g, 0..3): one AF float4 per row
  if (tid < 128) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = pd_unit(g, eu);
      const int col = (u >> 2) * 16 + 4 * q + (u & 3);  // biases / style terms come in lstm_cols order
      cst[q * 128 + tid] = a.l1_b[col] + (EMT && a.e_spk1 ? a.e_spk1[(long)em * 4 * PD_H + col] : 0.f);
      cst[(4 + q) * 128 + tid] = a.l2_b[col];
      cst[(8 + q) * 128 + tid] = a.GS[(long)em * 4 * PD_H + col];
    }
  }
  float c1 = 0.f, c2 = 0.f;  // cell states of (em, unit 4g+eu), threads < 128
  const int len = rowv ? a.lengths[b] : 0;
  const float va_k = a.va[16 * j + (lane & 15)];
  const float b2p = a.pre_b2[32 * j + (tid & 31)];
  for (int e = tid; e < CWN; e += PD_NT) cw[e] = 0.f;
  if (tid < TM) al[tid] = 0.f;
  if (tid < 32) ssa[tid] = 0.f;
  if (tid == 0) {
    si[0] = 0;
    si[4] = 0;
    si[8] = 0;
    sc[2] = 0.f;
  }
  f32x4 vals[8];  // values[b][32*(tid/64) + 4i + e][64j + tid%64]: valuesT is [B][E2][TM], 0 past T_in
  {
    const f32x4* V = reinterpret_cast<const f32x4*>(a.valuesT + ((long)(rowv ? b : 0) * PD_E2 + 64 * j + (tid & 63)) * TM +
                                                    32 * (tid >> 6));
#pragma unroll
    for (int i = 0; i < 8; ++i) vals[i] = V[i];
  }
  f32x4 loc[NI];  // location features of the next step (cum = 0)
#pragma unroll
  for (int i = 0; i < NI; ++i) loc[i] = zero4;
  f32x4 accC0 = zero4, accC1 = zero4;  // L1 context rows of the next step (context(-1) = 0)
  if constexpr (EMT) {  // the emotion block of step 0 (zero_state: refnet_spk alone), host-written at parity 1
    const float* XE = a.EMTx + 32 * PD_EQ;
    mm(pd_ld4(XE, (w * 2) * 64 + lane), pd_ld4(XE, (w * 2 + 1) * 64 + lane), w1e, accC0, accC1);
  }
  f32x4 q1a = zero4, q1b = zero4, q2a = zero4, q2b = zero4;  // this wave's Q partials of RG1, RG2
  const long BP = (long)a.B * PD_P;

  // Prenet (modules.py:346-357, dropout always on) of decoder step ts for row b, outputs
  // [32j, 32j+32).  Layer-1 work runs on threads 256..511 (position tid-256, AF-group column order
  // of the folded pre-activations) so wave 0 -- the poller -- never waits on the keep-bit loads.
  struct PrenetOps {
    float keep1, keep2;
    f32x4 w2p[4];  // W2[16*(tid/32) + 4i + e][32j + tid%32] (pre_w2t is [P][P] transposed; L2-resident)
  };
  auto prenet_keep = [&](int ts, int tid, float& k1, float& k2) {
    k1 = k2 = 0.f;
    if (rowv && ts < a.max_iters && tid >= 256) {
      const int pos = tid - 256;
      const int col = 16 * (pos >> 4) + ((pos >> 2) & 3) + 4 * (pos & 3);
      k1 = (float)a.masks[(long)ts * 2 * BP + (long)b * PD_P + col];
      if (pos < 32) k2 = (float)a.masks[((long)ts * 2 + 1) * BP + (long)b * PD_P + 32 * j + pos];
    }
  };
  auto prenet_ops = [&](float k1, float k2, int tid) {
    PrenetOps o;
    o.keep1 = k1;
    o.keep2 = k2;
    const f32x4* W2 = reinterpret_cast<const f32x4*>(a.pre_w2t + (long)(32 * j + (tid & 31)) * PD_P + 16 * (tid >> 5));
#pragma unroll
    for (int i = 0; i < 4; ++i) o.w2p[i] = W2[i];
    return o;
  };
  auto prenet = [&](const PrenetOps& o, auto pre1, int par, unsigned tag, int tid) {
    if (tid >= 256) {
      const int pos = tid - 256;
      const int col = 16 * (pos >> 4) + ((pos >> 2) & 3) + 4 * (pos & 3);  // af_group_col(pos)
      x1[col] = rowv ? (fmaxf(pre1(pos), 0.f) / 0.5f) * o.keep1 : 0.f;
      if (pos < 32) red[3072 + pos] = o.keep2;  // layer-2 keep bits -> the 32 output threads
    }
    __syncthreads();
    {
      const int k16 = tid >> 5;  // wave w: k16 = 2w (lanes 0..31), 2w + 1 (lanes 32..63)
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (!FL || i == 0) s += x1[16 * k16 + i] * o.w2p[i >> 2][i & 3];
      s += __shfl_xor(s, 32);
      if ((tid & 63) < 32) red[(tid >> 6) * 32 + (tid & 31)] = s;
    }
    __syncthreads();
    if (tid < 32) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += red[ww * 32 + tid];
      const int n = 32 * j + tid;
      const float out = rowv ? (fmaxf(v + b2p, 0.f) / 0.5f) * red[3072 + tid] : 0.f;
      pd_put(a.PREg + par * 32 * PD_P + af_idx(b, n), tag, out);
    }
  };

  // Recurrent tail half h (all 8 waves, K split 8 ways, k-groups 8w + 4h .. +4).  The zoned-state
  // recurrence RG(t+1) = h_z(t)·W_h = (1-z)·h_new(t)·W_h + z·RG(t) is linear in h_new, so every wave
  // keeps its own K-slice partial Q_w with RG = (1-z)·Σ_w Q_w:  Q_w(t+1) = z·Q_w(t) + h_new(t)·W_h
  // (its slice), in registers.  No reduction: the partials join the gate accumulators of stage A/B,
  // whose cross-wave reduction runs anyway.  The two halves sit in two hand-off windows.
  // Recurrent tail loads.  Only the RG2 tail of the F window (h2 of this step, all rows) checks the
  // tags: the other tails read values this work-group already depends on (RG1: the k-slice this wave
  // took in stage B; RG2 in the A window: h2 of step t-1, which every context, projection partial
  // and prenet granule of t-1 -- taken before stage A -- was computed from).
  auto rec_half = [&](int ph, const float* X, unsigned tb, const float* Wl, int h, f32x4& Qa, f32x4& Qb, int w,
                      int lane, bool check) {
    const f32x4* Wv = reinterpret_cast<const f32x4*>(Wl);
    f32x4 xv[8];
    const auto ix = [&](int i) { return ((8 * w + 4 * h + (i >> 1)) * 2 + (i & 1)) * 64 + lane; };
    if (check) {
      if (!pd_take4<8>(a, ph, X, ix, tb, xv, [] { return true; })) si[8] = 1;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = pd_ld4(X, ix(i));
    }
    if (h == 0) {
      Qa = a.zo * Qa;
      Qb = a.zo * Qb;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int sg = 8 * w + 4 * h + i;
      mm(xv[2 * i], xv[2 * i + 1], Wv[sg * 64 + lane], Qa, Qb);
    }
  };
  __syncthreads();
  // GO frame (helpers.py:136-138): frame 0 -> layer-1 pre-activation = b1
  {
    float k1, k2;
    prenet_keep(0, tid, k1, k2);
    prenet(prenet_ops(k1, k2, tid), [&](int pos) { return a.pre_b1[pos]; }, 0, 1u << 1, tid);
  }
  if (tid == 0) si[1] = 0;
  __syncthreads();

  for (int t = 0; t < a.max_iters; ++t) {
    const unsigned tg = t + 1;
    const int p = t & 1;
    const unsigned tb = pd_tb(t), tbp = pd_tb(t - 1);  // self-tag bits of steps t, t-1
    long long* const stp = (stp0 && t == a.stamp_step) ? stp0 : nullptr;
    // Thread indices re-derived from an opaque copy every step: otherwise every loop-invariant
    // LDS/global address of the body is hoisted out of the step loop and spilled.
    int tid = tid_, lane, w, em, eu;
    asm volatile("" : "+v"(tid));
    lane = tid & 63;
    w = tid >> 6;
    em = (tid >> 2) & 31;
    eu = tid & 3;
    PD_STAMP(0);
    if constexpr (!EMT) {  // diagnostic: the hardware XCD of this work-group (HW_REG_XCC_ID bits 3:0)
      if (stp && tid == 0) stp[g * 32 + 31] = __builtin_amdgcn_s_getreg(0x1814) & 15;
    }
    float keep1n, keep2n;  // prenet keep bits of step t+1, in flight during the whole step
    prenet_keep(t + 1, tid, keep1n, keep2n);
    // ================= A: LSTM layer 1 =================
    // prenet(t) of every row arrives as AF-ordered granules {tag = (t+1)<<1 | stop bit of the
    // producing row at t-1, value}; wave w takes k-groups 2w, 2w+1 = columns [32w, 32w+32), written
    // by the 32 work-groups of slice j = w, so the 8 waves together hear from all 256.
    f32x4 a0[2], a1[2];
    {
      const auto rp = __builtin_amdgcn_make_buffer_rsrc(a.PREg + p * 32 * PD_P, (short)0, 0x7fffffff, 0x00020000);
      unsigned sb[2] = {0u, 0u};  // stop bits of rows lane%16 and 16 + lane%16
      long long t0 = 0;
      for (unsigned spin = 0;; ++spin) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int fo = (((2 * w + i) * 2 + h) * 64 + lane) * 4;  // AF float index of the lane's float4
            const auto q0 = __builtin_amdgcn_raw_buffer_load_b128(rp, fo * 8, 0, 16);       // granules 0, 1
            const auto q1 = __builtin_amdgcn_raw_buffer_load_b128(rp, fo * 8 + 16, 0, 16);  // granules 2, 3
            f32x4 v = {__uint_as_float(q0[0]), __uint_as_float(q0[2]), __uint_as_float(q1[0]), __uint_as_float(q1[2])};
            ok = ok && (q0[1] >> 1) == tg && (q0[3] >> 1) == tg && (q1[1] >> 1) == tg && (q1[3] >> 1) == tg;
            if (h == 0) a0[i] = v;
            else a1[i] = v;
            if (i == 0) sb[h] = q0[1] & 1u;
          }
        if (__all(ok)) break;
        if ((spin & 31) == 0) {
          const long long now = __builtin_amdgcn_s_memrealtime();
          if (spin == 0) {
            t0 = now;
          } else if (__hip_atomic_load((pd_gi32*)(a.ctl + 2), PD_RLX) != 0 || now - t0 > PD_TIMEOUT) {
            if (lane == 0) {
              __hip_atomic_store((pd_gi32*)(a.ctl + 2), 1 + PD_F_PRE, PD_RLX);
              atomicMax(si + 1, 2);
            }
            break;
          }
        }
        for (int z = 0; z < a.poll_sleep; ++z) __builtin_amdgcn_s_sleep(1);
      }
      if (t > 0 && w == 0) {
        // stop rule of step t-1 (TacoTestHelper.next_inputs, helpers.py:40-59 + dynamic_decode):
        // every valid row rounds to 1; GTA stops at T_targets instead.  stop_at_any does not change it at
        // r = 1: TacoTestHelper reduces the batch axis first (reduce_all(finished, axis=0) over [B, r],
        // helpers.py:40-54), then any / all over the r frames of the step
        int dn;
        if (a.T_lim > 0) {
          dn = t >= a.T_lim;
        } else {
          const int r0 = lane & 15;
          const bool v0 = lane < 16 && r0 < a.B, v1 = lane < 16 && r0 + 16 < a.B;
          const unsigned long long f0 = __ballot(v0 && sb[0]), f1 = __ballot(v1 && sb[1]);
          const unsigned long long m0 = __ballot(v0), m1 = __ballot(v1);
          dn = a.stop_at_any == 2 ? 0 : (f0 == m0 && f1 == m1);
        }
        if (lane == 0 && dn) atomicMax(si + 1, 1);
      }
    }
    PD_STAMP(1);
    {
      // L1 context rows of t-1 (accumulated during the prenet hand-off) + this wave's RG1 partial
      f32x4 s0 = accC0 + a.one_m_zo * q1a, s1 = accC1 + a.one_m_zo * q1b;
#pragma unroll
      for (int i = 0; i < 2; ++i) mm(a0[i], a1[i], w1p[i], s0, s1);
      PD_STAMP(18);
      put_partials(s0, s1, red, w, lane);
      __syncthreads();
      PD_STAMP(19);
    }
    if (si[1]) {  // 1: the batch stopped at t-1 (every work-group decides alike); 2: a hand-off failed
      if (si[1] == 1 && g == 0 && tid == 0) {
        a.ctl[1] = t;
        a.ctl[0] = 1;
      }
      return;
    }
    if (tid < 128) {
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = em * 16 + 4 * q + eu;
        z[q] = (sum_partials<8>(red, idx) * KG_UNSCALE + ssa[em] * cst[(8 + q) * 128 + tid]) + cst[q * 128 + tid];
      }
      const float cn = sigm_fast(z[2] + 1.0f) * c1 + sigm_fast(z[0]) * tanh_rcp(z[1]);
      const float hn = sigm_fast(z[3]) * tanh_rcp(cn);
      c1 = a.one_m_zo * cn + a.zo * c1;
      pd_st_h4(a.H1x + p * 32 * PD_H, em, u0, hn, lane, PD_TAG_H1 ? tb : ~0u);
    }
    if constexpr (PD_TAG_H1) pd_hint_rep(a, 0, tg, tid);
    else pd_publish_rep(a, 0, tg, tid);
    PD_STAMP(2);
    if (t > 0) rec_half(PD_F_H2, a.H2x + (p ^ 1) * 32 * PD_H, tbp, sW2h, 1, q2a, q2b, w, lane, false);  // RG2(t), 2nd half
    PD_STAMP(3);
    // ================= B: LSTM layer 2 =================
    // wave w multiplies h1 units [128w, 128w+128) = the rows of producers [32w, 32w+32)
    if constexpr (!PD_TAG_H1)
      if (!pd_poll_rep(a, PD_F_H1, 0, 32 * w, tg, lane)) si[8] = 1;
    PD_STAMP(4);
    {
      const float* X = a.H1x + p * 32 * PD_H;
      f32x4 s0 = a.one_m_zo * q2a, s1 = a.one_m_zo * q2b;  // + this wave's RG2 partial
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 xv[8];
        const auto ix = [&](int i) { return ((8 * w + 4 * h + (i >> 1)) * 2 + (i & 1)) * 64 + lane; };
        if constexpr (PD_TAG_H1 == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) xv[i] = pd_ld4(X, ix(i));
        } else if constexpr (PD_TAG_H1 == 1) {
          if (!pd_take4<8>(a, PD_F_H1, X, ix, tb, xv, [&] { return pd_poll_rep(a, PD_F_H1, 0, 32 * w, tg, lane); }))
            si[8] = 1;
        } else {
          if (!pd_take4<8>(a, PD_F_H1, X, ix, tb, xv, [] { return true; })) si[8] = 1;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) mm(xv[2 * i], xv[2 * i + 1], w2i[4 * h + i], s0, s1);
      }
      PD_STAMP(16);
      put_partials(s0, s1, red, w, lane);
      __syncthreads();
      PD_STAMP(17);
      if (si[8]) return;
    }
    if (tid < 128) {
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = em * 16 + 4 * q + eu;
        z[q] = sum_partials<8>(red, idx) * KG_UNSCALE + cst[(4 + q) * 128 + tid];
      }
      const float cn = sigm_fast(z[2] + 1.0f) * c2 + sigm_fast(z[0]) * tanh_rcp(z[1]);
      const float hn = sigm_fast(z[3]) * tanh_rcp(cn);
      c2 = a.one_m_zo * cn + a.zo * c2;
      pd_st_h4(a.H2x + p * 32 * PD_H, em, u0, hn, lane, tb);
    }
    pd_hint_rep(a, 1, tg, tid);
    PD_STAMP(5);
    // issued ahead of the RG1 tail and the H2 wait (L2-resident: shared by the 32 rows of slice j):
    f32x4 wq[8];  // W_q[32*(tid/16) + 4i + e][16j + tid%16] (q_wt is [A][H])
    {
      const f32x4* Q = reinterpret_cast<const f32x4*>(a.q_wt + (long)(16 * j + (tid & 15)) * PD_H + 32 * (tid >> 4));
#pragma unroll
      for (int i = 0; i < 8; ++i) wq[i] = Q[i];
    }
    f32x4 kv[NI];  // keys[b][t0 + r][16j + lane%16], t0 = 16(w + 8i) + 4(lane/16): keysT is [B][A][TM]
    {
      const f32x4* K = reinterpret_cast<const f32x4*>(a.keysT + ((long)(rowv ? b : 0) * PD_A + 16 * j + (lane & 15)) * TM);
#pragma unroll
      for (int i = 0; i < NI; ++i) kv[i] = K[(w + 8 * i) * 4 + (lane >> 4)];
    }
    rec_half(PD_F_H1, a.H1x + p * 32 * PD_H, tb, sW1h, 0, q1a, q1b, w, lane, false);  // RG1(t+1) from h1_new(t), 1st half
    PD_STAMP(6);
    // ================= C: query slice + partial energies (attention.py:37-69, 186-201) =================
    // wave w: h2 units [128w, 128w+128) of row b (producers [32w, 32w+32)), tagged loads
    PD_STAMP(7);

    if (rowv) {
      const float* X = a.H2x + p * 32 * PD_H;
      // wave w reads exactly the h2 units [128w, 128w+128) its own lanes multiply: wave-local
      // exchange (LDS ops of one wave complete in order), one block barrier for the 8 wave partials
      float hv[2];
      if (!pd_take1<2>(a, PD_F_H2, X, [&](int i) { return af_idx(b, 128 * w + 64 * i + lane); }, tb, hv,
                       [&] { return pd_poll_rep(a, PD_F_H2, 1, 32 * w, tg, lane); }))
        si[8] = 1;
      red[128 * w + lane] = hv[0];
      red[128 * w + 64 + lane] = hv[1];
      __builtin_amdgcn_wave_barrier();
      {
        const int seg = tid >> 4;
        float s = 0.f;
        if constexpr (FL) {
          s = red[seg * 32];
          asm volatile("" ::"v"(wq[0]), "v"(wq[1]), "v"(wq[2]), "v"(wq[3]), "v"(wq[4]), "v"(wq[5]), "v"(wq[6]), "v"(wq[7]));
        } else {
#pragma unroll
          for (int ii = 0; ii < 32; ++ii) s += red[seg * 32 + ii] * wq[ii >> 2][ii & 3];
          s += __shfl_xor(s, 16);
          s += __shfl_xor(s, 32);
        }
        if (lane < 16) red[1024 + w * 16 + lane] = s;
      }
      __syncthreads();
      float qk = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) qk += red[1024 + ww * 16 + (lane & 15)];
      unsigned long long* E = a.Eg + (((long)p * 32 + b) * 8 + j) * TM;
      // after sum16 every lane of group q = lane/16 holds the energies of positions 4q + r; one
      // shuffle gathers position l (l < 16) of tile i on lane 16 i + l, so the 16 NI granules leave
      // as ONE store instruction of whole 128-B lines (not 4 NI stores of 4 lanes at a 32-B stride,
      // each its own fabric write)
      float sel[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float e4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          e4[r] = FL ? kv[i][r] + qk + loc[i][r] : sum16(va_k * tanh_rcp(kv[i][r] + qk + loc[i][r]));
        const int rr = lane & 3;
        sel[i] = rr == 0 ? e4[0] : rr == 1 ? e4[1] : rr == 2 ? e4[2] : e4[3];
      }
      const int src = ((lane >> 2) & 3) * 16 + (lane & 3);
      float vi[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) vi[i] = __shfl(sel[i], src);
      float vo = vi[0];
#pragma unroll
      for (int i = 1; i < NI; ++i) vo = (lane >> 4) == i ? vi[i] : vo;
      if (lane < 16 * NI) pd_put(E + (w + 8 * (lane >> 4)) * 16 + (lane & 15), tg, vo);
    }
    __syncthreads();  // red / qv reuse below
    if (si[8]) return;
    PD_STAMP(8);
    if (isproj) {  // projection partial, h2_new rows of this split (Architecture_wrappers.py:243-247)
      const float* X = a.H2x + p * 32 * PD_H;
      const int sg = 8 * pks + w;  // h2 units [128 pks + 16w, +16): producers [32 pks, 32 pks + 32)
      f32x4 s0 = zero4, s1 = zero4, xv[2];
      if (!pd_take4<2>(a, PD_F_H2, X, [&](int i) { return (sg * 2 + i) * 64 + lane; }, tb, xv,
                       [&] { return pd_poll_rep(a, PD_F_H2, 1, 32 * pks, tg, lane); }))
        si[8] = 1;
      mm(xv[0], xv[1], WPH[w * 64 + lane], s0, s1);
      reduce_waves_32x16<8>(s0, s1, red, G, w, lane, tid);
      if (isq) {  // emotion query: h2 rows are all of it -> granules for the emotion work-groups
        const int m = tid >> 4, col = tid & 15;
        pd_put(a.QEg + (((long)p * PD_KSP + pks) * 32 + m) * PD_EQ + 16 * (pn - PD_NTILE) + col, tg, G[tid]);
      } else {
        PPh[tid] = G[tid];
      }
    }
    // ================= D: softmax, cumulative alignments, context (attention.py:10-35, 202-227) ==========
    PD_STAMP(9);
    if (rowv) {
      const unsigned long long* E = a.Eg + ((long)p * 32 + b) * 8 * TM;
      // TM = 512: the values of positions [256 + 32 (tid/64), +32) of channel 64j + tid%64 for the
      // context below, in flight across the energy take and the softmax
      f32x4 vhi[TM == PD_TMAX ? 1 : 8];
      if constexpr (TM != PD_TMAX) {
        const f32x4* V = reinterpret_cast<const f32x4*>(a.valuesT + ((long)(rowv ? b : 0) * PD_E2 + 64 * j + (tid & 63)) * TM +
                                                        PD_TMAX + 32 * (tid >> 6));
#pragma unroll
        for (int i = 0; i < 8; ++i) vhi[i] = V[i];
      }
      if (tid == 0) si[5] = 1;
      __syncthreads();
      // waves 0..NWE-1 hold one energy per lane; max and sum as wave shuffles + one LDS exchange of
      // the wave results each
      float e = -INFINITY;
      if (tid < TM) {
        float ev[8];
        if (!pd_take<8>(a, PD_F_E, E, tid, TM, tg, tid < T, ev)) si[5] = 0;
        if (tid < T) {
          e = 0.f;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) e += ev[jj];
          if (a.constraint) {  // synthesis window (attention.py:202-215)
            const int pm = si[0], wn = a.win;
            bool masked;
            if (a.monotonic) masked = (tid < pm) || (tid >= pm + wn);
            else masked = (tid < pm - (wn / 2 + (wn % 2 != 0 ? 1 : 0))) || (tid >= pm + wn / 2);
            if (masked) e = -4294967296.0f;  // -2**32 + 1 in fp32
          }
          if (a.mask_encoder && tid >= len) e = -INFINITY;
        }
        const float mx = wave_max_dpp(e);
        if (lane == 0) red[w] = mx;
      }
      __syncthreads();
      if (!si[5]) return;
      float ex = 0.f;
      if (tid < TM) {
        float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        if constexpr (NWE == 8) mx = fmaxf(mx, fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7])));
        ex = tid < T ? __expf(e - mx) : 0.f;
        const float sum = wave_sum_dpp(ex);
        if (lane == 0) red[8 + w] = sum;
      }
      __syncthreads();
      PD_STAMP(21);
      if (tid < TM) {
        float den = (red[8] + red[9]) + (red[10] + red[11]);
        if constexpr (NWE == 8) den += (red[12] + red[13]) + (red[14] + red[15]);
        al[tid] = tid < T ? ex * __builtin_amdgcn_rcpf(den) : 0.f;
      }
      __syncthreads();
      if (tid < T) {
        const float cp = cw[15 + tid];
        cw[15 + tid] = a.cumulative ? al[tid] + cp : al[tid];
        if (j == 0 && a.align) a.align[((long)b * a.max_iters + t) * T + tid] = al[tid];  // step-major
      }
      if (w == 1) {  // max_att = argmax (ties -> first), Σ_{t<len} alignments
        float best = -INFINITY, ss = 0.f;
        int bi = 0x7fffffff;
        for (int i = lane; i < T; i += 64) {
          if (al[i] > best) {
            best = al[i];
            bi = i;
          }
          if (i < len) ss += al[i];
        }
        for (int o = 32; o > 0; o >>= 1) {
          const float ob = __shfl_xor(best, o);
          const int oi = __shfl_xor(bi, o);
          if (ob > best || (ob == best && oi < bi)) {
            best = ob;
            bi = oi;
          }
          ss += __shfl_xor(ss, o);
        }
        if (lane == 0) {
          si[0] = bi;
          sc[2] = ss;
        }
      }
      {
        const int c = tid & 63, ts = tid >> 6;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i)
          if (!FL || i == 0) s += al[ts * 32 + i] * vals[i >> 2][i & 3];
        if constexpr (FL) asm volatile("" ::"v"(vals[1]), "v"(vals[2]), "v"(vals[3]), "v"(vals[4]), "v"(vals[5]), "v"(vals[6]), "v"(vals[7]));
        if constexpr (TM != PD_TMAX) {
#pragma unroll
          for (int i = 0; i < 32; ++i) s += al[PD_TMAX + ts * 32 + i] * vhi[i >> 2][i & 3];
        }
        red[ts * 64 + c] = s;
      }
      __syncthreads();
      if (tid < 64) {
        float s = 0.f;
#pragma unroll
        for (int ts = 0; ts < 8; ++ts) s += red[ts * 64 + tid];
        pd_st(a.CTXx + p * 32 * PD_E2 + af_idx(b, 64 * j + tid), pd_tag(s, tb));
      }
      if (tid == 64 && j == 0) pd_st(a.SSx + p * 32 + b, pd_tag(sc[2], tb));
    } else {
      if (tid < 64) pd_st(a.CTXx + p * 32 * PD_E2 + af_idx(b, 64 * j + tid), pd_tag(0.f, tb));
      if (tid == 64 && j == 0) pd_st(a.SSx + p * 32 + b, pd_tag(0.f, tb));
    }
    if constexpr (EMT) {
      if (tid == 0) si[6] = 1;  // emotion-stage failure flag (read after barriers below)
    }
    pd_hint(a, PD_F_CTX, tg, tid);
    PD_STAMP(10);
    rec_half(PD_F_H1, a.H1x + p * 32 * PD_H, tb, sW1h, 1, q1a, q1b, w, lane, false);  // RG1(t+1), 2nd half
    // location features of step t+1: im2col(cum) · (W_conv·W_loc) on MFMA (attention.py:59-62)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int t0 = (w + 8 * i) * 16 + (lane & 15) + (lane >> 4);
      f32x4 l = zero4;
#pragma unroll
      for (int sg = 0; sg < 2; ++sg)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if constexpr (FL) asm volatile("" ::"v"(cw[t0 + 16 * sg + 4 * e]), "v"(swl[64 * sg + lane][e]));
          else l = __builtin_amdgcn_mfma_f32_16x16x4f32(cw[t0 + 16 * sg + 4 * e], swl[64 * sg + lane][e], l, 0, 0, 0);
      loc[i] = l;
    }
    // ================= E: projection partial, context rows =================
    if constexpr (EMT) {
      if (g >= PD_EG0) {  // emotion rows r0, r0+1 (Architecture_wrappers.py:228-240, multihead_attention.py:35-132)
        const int r0 = 2 * (g - PD_EG0);
        float* qe = red;         // [2][128] query
        float* sco = red + 256;  // [2][heads][Tv] scores -> weights
        float* vls = red + 256 + 2 * a.e_heads * a.e_Tv;  // [2][Tv][Dv] values of the two rows, when they fit
        const int nv = a.e_Tv * a.e_Dv;
        const bool vl = 256 + 2 * a.e_heads * a.e_Tv + 2 * nv <= 4096;
        // the value loads are issued first and stored to LDS after the query take, so the two memory
        // round trips overlap
        float vt[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int e = tid + PD_NT * u, rr = e >= nv, b2 = r0 + rr;
          vt[u] = (vl && e < 2 * nv && b2 < a.B) ? a.e_val[b2 * a.e_vbs + (e - rr * nv)] : 0.f;
        }
        {  // 4 of the 8 K-split partials per thread (threads 256.. take splits 4..7): few registers
          const int row = r0 + ((tid >> 7) & 1), col = tid & 127, hs = tid >> 8;
          float pv[PD_KSP / 2];
          if (!pd_take<PD_KSP / 2>(a, PD_F_QE, a.QEg + (((long)p * PD_KSP + 4 * hs) * 32 + row) * PD_EQ, col, 32 * PD_EQ,
                                   tg, true, pv))
            si[6] = 0;
          G[tid] = (pv[0] + pv[1]) + (pv[2] + pv[3]);
        }
        if (vl)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (tid + PD_NT * u < 2 * nv) vls[tid + PD_NT * u] = vt[u];
        __syncthreads();
        if (tid < 256) qe[tid] = (G[tid] + G[256 + tid]) * KG_UNSCALE + a.e_qrow[(r0 + (tid >> 7)) * PD_EQ + (tid & 127)];
        __syncthreads();
        PD_STAMP(22);
        if (!si[6]) return;
        const int HT = a.e_heads * a.e_Tv;
        {  // s = Σ_d normed_v·tanh(keys + q + attention_b): lane d of a 32-lane group per dim (dh <= 32),
           // 16 scores per pass of 512 threads, the keys of 4 passes loaded before their arithmetic
          // ('simple': V(tanh(W1 v + W2 q)) over 128 units, split into 4 x 32-unit partials with each
          // part's own V slice and no attention_b; the partials are summed below)
          const int dh = a.e_dh, d = tid & 31;
          const float vvd = d < dh && !a.e_simple ? a.e_vv[d] : 0.f, abd = d < dh && !a.e_simple ? a.e_ab[d] : 0.f;
          for (int s0 = 0; s0 < 2 * HT; s0 += 64) {
            float kx[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int sidx = s0 + (tid >> 5) + 16 * u;
              const int rr = sidx / HT, hh = (sidx % HT) / a.e_Tv, tv = sidx % a.e_Tv, b2 = r0 + rr;
              kx[u] = (sidx < 2 * HT && b2 < a.B && d < dh) ? a.e_ke[b2 * a.e_kbs + (long)tv * PD_EQ + hh * dh + d] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int sidx = s0 + (tid >> 5) + 16 * u;
              const int rr = sidx / HT, hh = (sidx % HT) / a.e_Tv;
              float x = 0.f;
              const float vv = a.e_simple ? a.e_vv[min(hh * dh + d, PD_EQ - 1)] : vvd;
              if (sidx < 2 * HT && d < dh) x = vv * tanh_rcp(kx[u] + qe[rr * PD_EQ + hh * dh + d] + abd);
              x = sum32_to_lane31(x);  // DPP: the 32-lane group's sum in its lane 31
              if (d == 31 && sidx < 2 * HT) sco[sidx] = x;
            }
          }
        }
        __syncthreads();
        if (a.e_simple) {  // one score per (row, t): the sum of the 4 unit-slice partials (in the head-0 slot)
          if (tid < 2 * a.e_Tv) {
            const int rr = tid / a.e_Tv, tv = tid - rr * a.e_Tv;
            float v = 0.f;
            for (int h = 0; h < a.e_heads; ++h) v += sco[(rr * a.e_heads + h) * a.e_Tv + tv];
            sco[rr * HT + tv] = v;
          }
          __syncthreads();
        }
        PD_STAMP(23);
        const int nsm = a.e_simple ? 2 : 2 * a.e_heads;  // softmax rows: (row, head), or one per row
        for (int pr = w; pr < nsm; pr += PD_NT / 64) {   // softmax over the attended rows, one
          float* r = sco + (a.e_simple ? pr * HT : pr * a.e_Tv);  // (row, head) per wave, lanes over t
          const float x = lane < a.e_Tv ? r[lane] : -INFINITY;     // (no mask: padded frames count)
          const float mx = wave_max_dpp(x);
          const float ex = lane < a.e_Tv ? __expf(x - mx) : 0.f;
          const float sum = wave_sum_dpp(ex);
          if (lane < a.e_Tv) r[lane] = ex * __builtin_amdgcn_rcpf(sum);
        }
        __syncthreads();
        PD_STAMP(30);
        {  // contexts, heads concatenated (_combine_heads): one AF float4 = k = i0 + 4c (c < 4, one head) of
           // one row per thread, stored as ONE 16-byte write-through store
          const int nq = a.e_KC / 4;
          // 'multihead': the contexts go to the dense blocks (CMB); 'style_tokens': they are the block (EMT)
          float* const cdst = a.e_dense ? a.CMBx + (long)p * 32 * a.e_KC : a.EMTx + (long)p * 32 * PD_EQ;
          const auto rc = __builtin_amdgcn_make_buffer_rsrc(cdst, (short)0, 0x7fffffff, 0x00020000);
          for (int e = tid; e < 2 * nq; e += PD_NT) {
            const int rr = e >= nq, q = e - rr * nq, b2 = r0 + rr;
            const int i0 = 16 * (q >> 2) + (q & 3), hh = i0 / a.e_Dv, d0 = i0 - hh * a.e_Dv;
            const float* al = sco + (rr * a.e_heads + hh) * a.e_Tv;
            const float* v = vl ? vls + rr * nv + d0 : a.e_val + min(b2, a.B - 1) * a.e_vbs + d0;
            float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
            for (int tv = 0; tv < a.e_Tv; ++tv) {
              const float wt = al[tv];
              const float* vr = v + tv * a.e_Dv;
              c0 = fmaf(wt, vr[0], c0);
              c1 = fmaf(wt, vr[4], c1);
              c2 = fmaf(wt, vr[8], c2);
              c3 = fmaf(wt, vr[12], c3);
            }
            const bool ok = b2 < a.B;
            const u32x4 dv = {__float_as_uint(ok ? c0 : 0.f), __float_as_uint(ok ? c1 : 0.f),
                              __float_as_uint(ok ? c2 : 0.f), __float_as_uint(ok ? c3 : 0.f)};
            __builtin_amdgcn_raw_buffer_store_b128(dv, rc, af_idx(b2, i0) * 4, 0, 16);  // sc1
          }
        }
        PD_STAMP(31);
        if (a.e_dense) pd_publish(a, PD_F_CMB, tg, tid);
        else pd_publish_rep(a, 2, tg, tid);
        PD_STAMP(24);
        if (a.e_simple) {  // [max_iters][B][1][T_v]
          for (int e = tid; e < 2 * a.e_Tv; e += PD_NT) {
            const int rr = e / a.e_Tv, b2 = r0 + rr;
            if (b2 < a.B) a.e_hist[((long)t * a.B + b2) * a.e_Tv + (e - rr * a.e_Tv)] = sco[rr * HT + e - rr * a.e_Tv];
          }
        } else {
          for (int e = tid; e < 2 * HT; e += PD_NT) {  // emotion alignments (output only: after the publish)
            const int rr = e / HT, b2 = r0 + rr;
            if (b2 < a.B) a.e_hist[((long)t * a.B + b2) * HT + (e - rr * HT)] = sco[e];
          }
        }
      } else if (isq && a.e_dense) {  // attn_emt dense (Architecture_wrappers.py:233-234): tile pn - PD_NTILE, K split pks
        if (!pd_block_wait(si + 6, [&] { return pd_poll(a, PD_F_CMB, PD_EG0, 1, 16, tg, 0, lane); })) return;
        PD_STAMP(25);
        const int nkg = a.e_KC / 128;  // k-groups per split
        if (w < nkg) {
          const float* X = a.CMBx + (long)p * 32 * a.e_KC;
          const int sg = pks * nkg + w;
          f32x4 s0 = zero4, s1 = zero4;
          mm(pd_ld4(X, (sg * 2) * 64 + lane), pd_ld4(X, (sg * 2 + 1) * 64 + lane), wdf, s0, s1);
          put_partials(s0, s1, red, w, lane);
        }
        __syncthreads();
        {
          const int m = tid >> 4, col = tid & 15;
          float v = 0.f;
          for (int ww = 0; ww < nkg; ++ww) v += red[ww * 512 + tid];
          pd_put(a.EOg + (((long)p * PD_KSP + pks) * 32 + m) * PD_EQ + 16 * (pn - PD_NTILE) + col, tg, v);
        }
        __syncthreads();
        PD_STAMP(26);
      }
    }
    if (isproj && !isq) {
      PD_STAMP(11);
      if (w < 4) {  // context channels [64 pks + 16w, +16): slice j = pks, producers [32 pks, 32 pks + 32)
        const float* X = a.CTXx + p * 32 * PD_E2;
        const int sg = 4 * pks + w;
        f32x4 s0 = zero4, s1 = zero4, xv[2];
        if (!pd_take4<2>(a, PD_F_CTX, X, [&](int i) { return (sg * 2 + i) * 64 + lane; }, tb, xv,
                         [&] { return pd_poll(a, PD_F_CTX, 32 * pks, 1, 32, tg, 0, lane); }))
          si[8] = 1;
        mm(xv[0], xv[1], wpc, s0, s1);
        put_partials(s0, s1, red, w, lane);
      }
      __syncthreads();
      if (si[8]) return;
      {
        const int m = tid >> 4, col = tid & 15;
        pd_put(a.PPg + (((long)p * PD_KSP + pks) * 32 + m) * PD_NPF + 16 * pn + col, tg, sum_partials<4>(red, tid) + PPh[tid]);
      }
      __syncthreads();  // red / PPh are reused by the next tail
      PD_STAMP(12);
    }
    // ================= F: frame / stop (modules.py:392-448), prenet of step t+1 =================
    rec_half(PD_F_H2, a.H2x + p * 32 * PD_H, tb, sW2h, 0, q2a, q2b, w, lane, true);  // RG2(t+1) from h2_new(t), 1st half
    PD_STAMP(13);
    int stopbit = 0;
    if (tid == 0) si[5] = 1;
    __syncthreads();  // also: every proj work-group's PPh / red reads of stage E are done
    {
      // Every work-group -- padding rows too -- takes its row's partials: seeing all 176 producers
      // is what orders the context slices of step t before the L1 context rows read after F.
      if (tid < 384) {  // waves 0..5: the 352 projection columns of row b, 8 K-split partials each
        float pv[PD_KSP];
        const bool act = tid < PD_NPF;
        if (!pd_take<PD_KSP>(a, PD_F_PP, a.PPg + ((long)p * PD_KSP * 32 + b) * PD_NPF, act ? tid : 0, 32 * PD_NPF,
                             tg, act, pv))
          si[5] = 0;
        if (act && rowv) {
          float v = 0.f;
#pragma unroll
          for (int ks = 0; ks < PD_KSP; ++ks) v += pv[ks];
          red[tid] = (v * KG_UNSCALE + sc[2] * a.PS[(long)b * PD_NPF + tid]) + a.proj_b[tid];
        }
      }
      __syncthreads();
      if (!si[5]) return;
      PD_STAMP(20);
    }
    if (rowv) {
      const float sv = sigm(red[a.nm]);
      if (j == 0) {
        if (tid < a.nm) a.frames[((long)b * a.max_iters + t) * a.nm + tid] = red[tid];
        if (tid == a.nm) a.stop[(long)b * a.max_iters + t] = sv;
      }
      stopbit = rintf(sv) == 1.0f;
    }
    const PrenetOps pops = prenet_ops(keep1n, keep2n, tid);  // W2 slice: L2-resident
    if (t + 1 < a.max_iters) {
      if (a.TP1) {  // GTA (TacoTrainingHelper): the next input is the teacher frame t
        const float* tp = a.TP1 + ((long)b * a.T_lim + min(t, a.T_lim - 1)) * PD_P;
        prenet(pops, [&](int pos) { return tp[pos]; }, p ^ 1, ((tg + 1) << 1) | (unsigned)stopbit, tid);
      } else {  // free running: frame t through the folded layer-1 columns of the projection
        prenet(pops, [&](int pos) { return red[PD_NPJ + pos]; }, p ^ 1, ((tg + 1) << 1) | (unsigned)stopbit, tid);
      }
    }
    __syncthreads();  // red reuse by stage A
    PD_STAMP(14);
#ifdef PD_XSTAMP
    if constexpr (!EMT) {  // diagnostic build: how long the stores still in flight at 14 take to drain
      if (stp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PD_STAMP(30);
      }
    }
#endif
    if constexpr (EMT) {
      if (g >= PD_EG0 && a.e_dense) {  // dense partials of rows r0, r0+1 -> the next step's emotion block (+ refnet_spk),
                          // after this work-group's own prenet hand-off
        const int r0 = 2 * (g - PD_EG0);
        {
          const int row = r0 + ((tid >> 7) & 1), col = tid & 127, hs = tid >> 8;
          float pv[PD_KSP / 2];
          if (!pd_take<PD_KSP / 2>(a, PD_F_EO, a.EOg + (((long)p * PD_KSP + 4 * hs) * 32 + row) * PD_EQ, col, 32 * PD_EQ,
                                   tg, true, pv))
            si[6] = 0;
          G[tid] = (pv[0] + pv[1]) + (pv[2] + pv[3]);
        }
        __syncthreads();
        if (tid < 256) {
          const int row = r0 + (tid >> 7), col = tid & 127;
          float o = (G[tid] + G[256 + tid]) * KG_UNSCALE + a.e_bd[col];
          if (a.e_spk && row < a.B) o += a.e_spk[row * PD_EQ + col];
          pd_st(a.EMTx + p * 32 * PD_EQ + af_idx(row, col), row < a.B ? o : 0.f);
        }
        PD_STAMP(27);
        pd_publish_rep(a, 2, tg, tid);
        PD_STAMP(28);
        if (!si[6]) return;
      }
    }
    {  // L1 context rows of step t+1 and the style scales (tagged loads: every context slice of t was
       // taken by a projection block before its PP partial, so the values have normally landed)
      const float* XC = a.CTXx + p * 32 * PD_E2;
      accC0 = zero4;
      accC1 = zero4;
      f32x4 xv[8];  // wave w: channels [64w, 64w + 64) = slice j = w, producers [32w, 32w + 32)
      if (!pd_take4<8>(a, PD_F_CTX, XC, [&](int i) { return ((4 * w + (i >> 1)) * 2 + (i & 1)) * 64 + lane; }, tb, xv,
                       [&] {
                         if constexpr (!EMT) {  // diagnostic: when wave w's optimistic context load missed
                           if (stp && lane == 0) stp[g * 32 + 22 + w] = __builtin_amdgcn_s_memrealtime();
                         }
                         return pd_poll(a, PD_F_CTX, 32 * w, 1, 32, tg, 0, lane);
                       }))
        si[8] = 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) mm(xv[2 * i], xv[2 * i + 1], w1c[i], accC0, accC1);
      if (w == 0) {  // Σ_{t<len} align of every row (written by the j = 0 work-groups, producers [0, 32))
        float sv[1];
        if (!pd_take1<1>(a, PD_F_CTX, a.SSx + p * 32, [&](int) { return lane & 31; }, tb, sv,
                         [&] { return pd_poll(a, PD_F_CTX, 0, 1, 32, tg, 0, lane); }))
          si[8] = 1;
        if (lane < 32) ssa[lane] = sv[0];
      }
    }
    if constexpr (EMT) {  // the emotion block of step t joins the next step's LSTM-1 input (wave w: k-group w)
      if (!pd_block_wait(si + 6, [&] { return pd_poll_rep(a, PD_F_EMT, 2, PD_EG0, tg, lane, 16); })) return;
      PD_STAMP(29);
      const float* XE = a.EMTx + p * 32 * PD_EQ;
      mm(pd_ld4(XE, (w * 2) * 64 + lane), pd_ld4(XE, (w * 2 + 1) * 64 + lane), w1e, accC0, accC1);
    }
    PD_STAMP(15);
  }
  if (g == 0 && tid == 0) {
    a.ctl[1] = a.max_iters;
    a.ctl[0] = 1;
  }
}

size_t pd_lds_bytes() { return sizeof(float) * (size_t)PD_LDS_FLOATS; }

bool pd_device_ok(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  if (prop.multiProcessorCount < PD_NB) return false;
  for (const void* k : {reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX, false>),
                        reinterpret_cast<const void*>(k_decode_persist<true, PD_TMAX, false>),
                        reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX_LONG, false>),
                        reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX, true>)})
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pd_lds_bytes()) != hipSuccess)
      return false;
  int nb = 0, ne = 0, nl = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_decode_persist<false, PD_TMAX, false>, PD_NT, pd_lds_bytes()) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&ne, k_decode_persist<true, PD_TMAX, false>, PD_NT, pd_lds_bytes()) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nl, k_decode_persist<false, PD_TMAX_LONG, false>, PD_NT, pd_lds_bytes()) !=
          hipSuccess)
    return false;
  return nb >= 1 && ne >= 1 && nl >= 1;
}

// Cooperative launch: the runtime guarantees every one of the PD_NB work-groups is resident at
// once (or fails the launch) -- the spin-waits of the hand-offs depend on it, and a plain launch
// could be starved of CUs by a concurrent kernel on another stream or context.
void pd_launch(const PdArgs& a, hipStream_t s, bool emt, int tm) {
  TT2_CHECK(tm == PD_TMAX || (tm == PD_TMAX_LONG && !emt), TT2_ERR_INVALID_ARG, "persistent decoder: unsupported geometry");
  TT2_CHECK(a.T_in >= 1 && a.T_in <= tm, TT2_ERR_INVALID_ARG, "persistent decoder: T_in outside the kernel's range");
  PdArgs arg = a;
  void* params[] = {&arg};
  static const bool floor_env = [] {  // diagnostic: the arithmetic-free floor instance (see FL)
    const char* e = std::getenv("TT2_PD_FLOOR");
    return e && e[0] == '1';
  }();
  const void* k = emt ? reinterpret_cast<const void*>(k_decode_persist<true, PD_TMAX, false>)
                  : tm != PD_TMAX ? reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX_LONG, false>)
                  : floor_env     ? reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX, true>)
                                  : reinterpret_cast<const void*>(k_decode_persist<false, PD_TMAX, false>);
  TT2_HIP(launch_persistent(k, dim3(PD_NB), dim3(PD_NT), params, (unsigned)pd_lds_bytes(), s));
}

}  // namespace tt2
