// Self-attention (flash-style, head dim 64) forward / backward and the folded 2-key
// cross-attention of the UNet's Transformer2DModel blocks (gfx950, MFMA 32x32x16 bf16).
//
// Layouts: qkv [nb*T][ld] bf16 with q | k | v column blocks (head h at column h*64 of each block),
// o [nb*T][ldo], lse [nb][heads][T] fp32 (natural log of sum exp(q.k/8)).
// The forward keeps S^T = K Q^T in registers (query on the lane), so softmax row statistics are
// lane-local; P feeds the P.V MFMA straight from the accumulator (O^T = V^T P^T) with V^T fragments
// from ds_read_b64_tr_b16.  The backward is split into a dK/dV kernel (keys resident per wave,
// sweeping queries) and a dQ kernel (queries resident, sweeping keys): deterministic, no atomics.
#include <type_traits>

#include "common.h"
#include <stdlib.h>
#include "../../include/dcamd.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

// raw v_exp_f32: exp2f() wraps it in a denormal-range fix-up (cmp/cndmask/add/ldexp, ~6 VALU per
// call), pure overhead for softmax weights, where results below 2^-126 may flush to zero
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
constexpr int KSTR = 72;   // row stride (elements) of row-read tiles: 144 B, conflict-free ds_read_b128
constexpr int VSTR = 96;   // row stride of tr-read-only tiles: 192 B, conflict-free ds_read_b64_tr_b16

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((DC_LDS bf16x4*)(p));
}

// A-operand (rows = column dim d of a row-major [key][d] LDS tile) with the permuted k order that
// matches an accumulator used as B operand: element j <-> key 16*s + 8*(j>>2) + 4*hh + (j&3).
__device__ __forceinline__ bf16x8 trans_frag(const bf16* tile, int stride, int key_base, int col_base, int lane) {
  const int g = lane >> 4, i = lane & 15, hh = lane >> 5;
  const int qq = i >> 2, pp = i & 3;
  const int col = col_base + 16 * (g & 1) + 4 * pp;
  const int k0 = key_base + 4 * hh + qq;
  bf16x4 lo = tr_read(tile + k0 * stride + col);
  bf16x4 hi = tr_read(tile + (k0 + 8) * stride + col);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__device__ __forceinline__ bf16x8 acc_to_frag(const f32x16& a, int half) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * half + j];
  return r;
}

__device__ __forceinline__ bf16x8 load_row8(const bf16* p, bool ok, float scale) {
  bf16x8 v;
  if (ok) {
    v = *reinterpret_cast<const bf16x8*>(p);
    if (scale != 1.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * scale);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)0.0f;
  }
  return v;
}

// stage a [64 rows][64 cols] bf16 tile (rows r0.., column offset col) into LDS with `stride`, by NT threads
// (t = 0..NT-1): 512 16-B pieces, PPT per thread
template <int NT>
constexpr int ppt() { return (512 + NT - 1) / NT; }

template <int NT>
__device__ __forceinline__ void stage_load(const bf16* base, long ld, int r0, int rows_total, int col,
                                           uint4 (&reg)[ppt<NT>()], int t) {
#pragma unroll
  for (int i = 0; i < ppt<NT>(); ++i) {
    const int p = t + NT * i;
    const int row = p >> 3, piece = p & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (p < 512 && r0 + row < rows_total)
      v = *reinterpret_cast<const uint4*>(base + (long)(r0 + row) * ld + col + piece * 8);
    reg[i] = v;
  }
}
template <int NT>
__device__ __forceinline__ void stage_store(bf16* tile, int stride, const uint4 (&reg)[ppt<NT>()], float scale,
                                            int t) {
#pragma unroll
  for (int i = 0; i < ppt<NT>(); ++i) {
    const int p = t + NT * i;
    if (p >= 512) break;
    const int row = p >> 3, piece = p & 7;
    uint4 v = reg[i];
    if (scale != 1.0f) {
      bf16x8 b = *reinterpret_cast<bf16x8*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = (bf16)((float)b[j] * scale);
      v = *reinterpret_cast<uint4*>(&b);
    }
    *reinterpret_cast<uint4*>(tile + row * stride + piece * 8) = v;
  }
}

// ---------------------------------------------------------------- LDS-DMA tiles (swizzled, unpadded)
// K / V / Q / dO tiles are [64 rows][64 bf16] = 128-B rows written by buffer_load_dwordx4 ... lds.
// The 16-B chunk c of row r lives at chunk c ^ tsw(r): conflict-free for the ds_read_b128 fragment
// reads (32 rows, one chunk per lane group) and for the ds_read_b64_tr_b16 transposed reads (rows
// k0..k0+3 / +8, 8-B pieces of 32 columns).
constexpr int kOOB = (int)0x80000000u;  // out-of-range buffer offset: the DMA writes zeros
constexpr int TILE_B = 64 * 128;

__device__ __forceinline__ int tsw(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int tile_off(int r, int c) { return r * 128 + (((c >> 3) ^ tsw(r)) << 4) + (c & 7) * 2; }

__device__ __forceinline__ bf16x8 row_frag(const char* tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(tile + row * 128 + ((chunk ^ tsw(row)) << 4));
}

// byte offsets of a lane's two tr_b16 reads for trans_frag_sw(key_base, col_base): loop-invariant,
// so kernels precompute them once (the swizzle arithmetic would otherwise be VALU in every tile)
struct TrOff {
  int lo, hi;
};
__device__ __forceinline__ TrOff tr_off(int key_base, int col_base, int lane) {
  const int g = lane >> 4, i = lane & 15, hh = lane >> 5;
  const int col = col_base + 16 * (g & 1) + 4 * (i & 3);
  const int k0 = key_base + 4 * hh + (i >> 2);
  return TrOff{tile_off(k0, col), tile_off(k0 + 8, col)};
}
__device__ __forceinline__ bf16x8 trans_frag_at(const char* tile, TrOff o) {
  bf16x4 lo = tr_read(reinterpret_cast<const bf16*>(tile + o.lo));
  bf16x4 hi = tr_read(reinterpret_cast<const bf16*>(tile + o.hi));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
__device__ __forceinline__ int row_off(int row, int chunk) { return row * 128 + ((chunk ^ tsw(row)) << 4); }

// Transposed fragments by inline-asm ds_read_b64_tr_b16, waited for explicitly (lgkm_wait).  Issued
// through the builtin, the read carries no alias scope, so the compiler's waitcnt pass assumes it may
// alias every LDS-DMA in flight and puts a vmcnt(0) in front of it -- draining the ring's prefetch of
// the next tiles on every tile.  addr: 32-bit LDS address of the lane's row piece; IMM: byte offset.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(unsigned long)((DC_LDS const char*)(p));
}
template <int IMM>
__device__ __forceinline__ bf16x8 trans_frag_nw(unsigned lo, unsigned hi) {
  bf16x4 a, b;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(a) : "v"(lo), "n"(IMM));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(b) : "v"(hi), "n"(IMM));
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
// wait until at most N LDS ops are outstanding; the fragments are operands so no use moves above it
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a, bf16x8& b, bf16x8& c, bf16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}

// transposed A-operand fragment from a swizzled tile (same element order as trans_frag)
__device__ __forceinline__ bf16x8 trans_frag_sw(const char* tile, int key_base, int col_base, int lane) {
  const int g = lane >> 4, i = lane & 15, hh = lane >> 5;
  const int qq = i >> 2, pp = i & 3;
  const int col = col_base + 16 * (g & 1) + 4 * pp;
  const int k0 = key_base + 4 * hh + qq;
  bf16x4 lo = tr_read(reinterpret_cast<const bf16*>(tile + tile_off(k0, col)));
  bf16x4 hi = tr_read(reinterpret_cast<const bf16*>(tile + tile_off(k0 + 8, col)));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, 0x7fffffff,
                                           0x00020000);
}
// (the builtin exists only in the device pass; unguarded it silently drops the host launch stub)
__device__ __forceinline__ void buf_load_lds16(__amdgpu_buffer_rsrc_t r, DC_LDS char* dst, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
#endif
}
__device__ __forceinline__ void buf_load_lds4(__amdgpu_buffer_rsrc_t r, DC_LDS char* dst, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 4, voff, soff, 0, 0);
#endif
}

// one 64-row tile by the NT threads of a split: 512 pieces of 16 B, piece p = lt + NT i, one LDS-DMA
// wave-instruction per 64 consecutive pieces; the source offset of each piece is fixed, the tile's
// first row rides in soffset, rows >= T read zero
template <int NT>
struct TileDma {
  static constexpr int PPT = (512 + NT - 1) / NT;
  static constexpr int MIN_INSTR = 512 / NT;  // instructions per tile issued by every wave (>=)
  int voff[PPT], prow[PPT];
  __device__ __forceinline__ void init(int lt, int ld) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = lt + NT * i, r = p >> 3;
      prow[i] = r;
      voff[i] = r * ld * 2 + (((p & 7) ^ tsw(r)) << 4);
    }
  }
  // (wave index and soffset go through readfirstlane: derived from threadIdx, the compiler would
  // otherwise treat them as divergent and waterfall every buffer access)
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* tile, int r0, int T, int ld, int lt) {
    const int wv = __builtin_amdgcn_readfirstlane(lt >> 6);
    const int soff = __builtin_amdgcn_readfirstlane(r0 * ld * 2);
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int first = 64 * wv + NT * i;
      if (first < 512) buf_load_lds16(rs, (DC_LDS char*)tile + first * 16, r0 + prow[i] < T ? voff[i] : kOOB, soff);
    }
  }
};

template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The ring's per-tile barrier.  The caller's counted vm_wait_n has landed this wave's pieces of the tile; the barrier
// makes every wave's pieces visible, and the lgkmcnt(0) ahead of it retires this wave's reads of the stage the next
// DMA overwrites.  No workgroup fence: __syncthreads() is a release fence as well, lowered with a vmcnt(0) that also
// waits for the LDS-DMA of the LATER tiles, i.e. drains the ring's prefetch at every tile.
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct AttnSK {
  float* slab;     // [G * spb slots][QW waves][NV values][64 lanes] fp32 partials
  int* counters;   // one per key- / query-block (global index), zero between launches
  long U;          // units: blocks x tiles swept
  int G, spb;      // blocks of the launch, slab slots per block
};

__device__ __forceinline__ long sk_start(const AttnSK& sk, long b) { return b * sk.U / sk.G; }

// the block whose range holds unit x
__device__ __forceinline__ long sk_block_of(const AttnSK& sk, long x) {
  long b = x * sk.G / sk.U;
  while (b + 1 < sk.G && sk_start(sk, b + 1) <= x) ++b;
  while (b > 0 && sk_start(sk, b) > x) --b;
  return b;
}

// Partial hand-off of NV accumulator values per lane for block-unit `bi` (global key- / query-block index,
// ntile tiles) swept by this block in segment `seg`.  Returns true in the block that must write the result,
// with v holding the ordered sum of every covering block's partial.
template <int QW, int NV, bool SUM = true>
__device__ __forceinline__ bool sk_handoff(const AttnSK& sk, char* smem, long bi, int ntile, int seg,
                                           float (&v)[NV]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long b = blockIdx.x;
  float* mine = sk.slab + (((b * sk.spb + seg) * QW + wid) * NV) * 64 + lane;
#pragma unroll
  for (int e = 0; e < NV; ++e) __hip_atomic_store(mine + e * 64, v[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long x0 = bi * ntile, x1 = x0 + ntile - 1;
  const long bf = sk_block_of(sk, x0), bl = sk_block_of(sk, x1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int* s_last = reinterpret_cast<int*>(smem);   // the ring is idle here
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(sk.counters + bi, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (int)(bl - bf);
    if (last) __hip_atomic_store(sk.counters + bi, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = last;
  }
  __syncthreads();
  const bool last = *s_last;
  __syncthreads();   // the next segment's LDS-DMA may land on the flag
  if (!last) return false;
  if constexpr (!SUM) return true;   // the caller folds the partials itself
#pragma unroll
  for (int e = 0; e < NV; ++e) v[e] = 0.0f;
  for (long bb = bf; bb <= bl; ++bb) {
    const long sg = bi - sk_start(sk, bb) / ntile;   // segment index of this block-unit in block bb
    const float* src = sk.slab + (((bb * sk.spb + sg) * QW + wid) * NV) * 64 + lane;
    float t[NV];
#pragma unroll
    for (int e = 0; e < NV; ++e) t[e] = __hip_atomic_load(src + e * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int e = 0; e < NV; ++e) v[e] += t[e];
  }
  return true;
}

// walk this block's stream-K range one block-unit segment at a time (units: nblk_units x ntile)
template <typename F>
__device__ __forceinline__ void sk_walk(const AttnSK& sk, int ntile, F&& seg_fn) {
  const long b = blockIdx.x;
  long u = sk_start(sk, b);
  const long uend = sk_start(sk, b + 1);
  const long first = u / ntile;
  while (u < uend) {
    const long bi = u / ntile;
    const int i0 = (int)(u - bi * ntile);
    const int i1 = (int)min((long)ntile, i0 + (uend - u));
    seg_fn(bi, i0, i1 - i0, (int)(bi - first));
    u += i1 - i0;
  }
}

// max of three without the IEEE-mode canonicalisation fmaxf gets (one v_max_f32 x, x, x per operand): the
// softmax inputs are MFMA results, NaN-free by construction
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// max over the two lanes of a row (lane l and l ^ 32) by v_permlane32_swap (no LDS round trip)
__device__ __forceinline__ float rowmax_pair(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3_raw(__uint_as_float(r[0]), __uint_as_float(r[1]), x);
}
__device__ __forceinline__ float rowsum_pair(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ------------------------------------------------------------------------------ forward
// KS key-splits per block: waves QW p .. QW p + QW - 1 sweep the p-th contiguous range of key tiles
// for the same 32 QW queries, then the partial (m, l, O) are merged through LDS in a fixed order.
// K / V tiles stream through an S-deep LDS-DMA ring per split (one barrier per tile).
constexpr int FWD_S = 3;
constexpr float FWD_TAU = 8.0f;  // lazy-rescale slack (natural-log units of the scaled scores)
constexpr float FWD_SUM_TAU = 2980.9579870417283f;   // e^FWD_TAU: the row-sum form of the same bound
template <int QW, int KS>
struct FwdLds {
  static constexpr int STAGE = 2 * TILE_B;                      // K + V
  static constexpr int RING = KS * FWD_S * STAGE;
  static constexpr int RED = (KS - 1) * QW * 34 * 64 * 4;
  static constexpr int BYTES = RING > RED ? RING : RED;
};

template <int QW, int KS>
__device__ __forceinline__ void fwd_segment(char* smem, const bf16* qkv, int ld, int T, int heads, bf16* o, int ldo,
                                            float* lse, int qbk, int h, int n, int t0, int tcount) {
  constexpr int NT = 64 * QW;
  constexpr int S = FWD_S;
  constexpr int STAGE = FwdLds<QW, KS>::STAGE;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int part = threadIdx.x / NT, wid = (threadIdx.x >> 6) - part * QW;
  const int lt = threadIdx.x - part * NT;
  char* ring = smem + part * S * STAGE;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const int my_q = qbk * (32 * QW) + wid * 32 + (lane & 31);
  const bool qok = my_q < T;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_row8(base + (long)my_q * ld + h * 64 + 16 * s + 8 * hh, qok, 0.125f);

  float m = -INFINITY, l = 0.0f;
  f32x16 oacc[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[db][r] = 0.0f;

  const int per = (tcount + KS - 1) / KS;
  const int tb = t0 + part * per;
  const int mine = max(0, min(t0 + tcount, tb + per) - tb);
  const __amdgpu_buffer_rsrc_t rk = buf_rsrc(base + C + h * 64);
  const __amdgpu_buffer_rsrc_t rv = buf_rsrc(base + 2 * C + h * 64);
  TileDma<NT> dma;
  dma.init(lt, ld);
  auto issue = [&](int i) __attribute__((always_inline)) {
    char* st = ring + (i % S) * STAGE;
    dma.issue(rk, st, (tb + i) * 64, T, ld, lt);
    dma.issue(rv, st + TILE_B, (tb + i) * 64, T, ld, lt);
  };
  constexpr int PER_TILE = 2 * TileDma<NT>::MIN_INSTR;  // LDS-DMA instructions per stage, every wave
  // per-lane LDS offsets of the K rows and LDS addresses of the V^T pieces for key half b = 0 / k-slice s = 0: the
  // swizzle phase depends on row bits 1..3 only, so key half b (+32 rows) and k-slice s (+16 rows) -- like the ring
  // stage -- are immediate offsets (4096 b, 2048 s bytes), and only these 4 + 4 registers stay live
  int koff[4];
  unsigned va[2][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) koff[s] = row_off(lane & 31, 2 * s + hh);
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    const TrOff o = tr_off(0, 32 * db, lane);
    va[db][0] = lds_addr(ring) + o.lo;
    va[db][1] = lds_addr(ring) + o.hi;
  }
  for (int i = 0; i < 2 && i < mine; ++i) issue(i);   // the DMA runs two tiles ahead
  f32x16 sacc[2];
  // S = K Q^T of tile i (ring stage ST: compile-time, the ds_read offsets are immediates)
  auto phase_s = [&](auto STC) __attribute__((always_inline)) {
    constexpr int ST = decltype(STC)::value;
    const char* kt_s = ring + ST * STAGE;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[b][r] = 0.0f;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        sacc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            *reinterpret_cast<const bf16x8*>(kt_s + 4096 * b + koff[s]), qf[s], sacc[b], 0, 0, 0);
    }
  };
  // online softmax of tile i (in sacc): updates (m, l), rescales O when the reference max moves, and returns P as the
  // four bf16 B-operand fragments of the P.V product
  auto phase_sm = [&](int i, bf16x8 (&pf)[4]) __attribute__((always_inline)) {
    const int kt = tb + i;
    // online softmax in raw score units; exp2 with log2(e) folded into one FMA per score;
    // keys beyond T exist only in the last tile; O is rescaled only when some row max grew
    if ((kt + 1) * 64 > T) {
      asm volatile("" ::: "memory");  // keep this a branch: if-converted it costs ~60 VALU per tile
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 64 + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key >= T) sacc[b][r] = -INFINITY;
        }
    }
    // row max: four independent v_max3 chains over the lane's 32 scores (raw v_max3: no canonicalising fmaxf on
    // the MFMA results, and no 32-deep serial chain), then the row's other lane half by v_permlane32_swap
    float mc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int b = c >> 1, r0 = 8 * (c & 1);
      float t = max3_raw(sacc[b][r0], sacc[b][r0 + 1], sacc[b][r0 + 2]);
      t = max3_raw(t, sacc[b][r0 + 3], sacc[b][r0 + 4]);
      t = max3_raw(t, sacc[b][r0 + 5], sacc[b][r0 + 6]);
      mc[c] = max3_raw(t, sacc[b][r0 + 7], sacc[b][r0 + 7]);
    }
    const float mx = rowmax_pair(max3_raw(max3_raw(mc[0], mc[1], mc[2]), mc[3], mc[3]));
    // lazy rescale: the reference max moves only when a row max exceeds it by more than FWD_TAU, so
    // weights stay <= e^FWD_TAU (exact in fp32 / bf16 relative terms; O and l share the reference)
    if (__any(mx > m + FWD_TAU)) {
      const float mnew = fmaxf(m, mx);
      const float alpha = fast_exp2((m - mnew) * LOG2E);
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] *= alpha;
      l *= alpha;
      m = mnew;
    }
    // row sums in fp32 from the unrounded weights: the LSE the backward recomputes P from must not carry
    // P's bf16 rounding (a sum of bf16 P, e.g. on the MFMA pipe, is off by up to ~4e-3 in the LSE on
    // peaked rows and biases the guidance gradient: tools/attn_acc.py, profiles/r02m)
    // (four partial sums: independent add chains, summed in a fixed order)
    const float ml = m * LOG2E;
    float ps[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = fast_exp2(fmaf(sacc[b][r], LOG2E, -ml));
        sacc[b][r] = pv;
        ps[r & 3] += pv;
      }
    l += (ps[0] + ps[1]) + (ps[2] + ps[3]);
#pragma unroll
    for (int s = 0; s < 4; ++s) pf[s] = acc_to_frag(sacc[s >> 1], s & 1);
  };
  // O += P V, V^T fragments of ring stage ST: two k-slices in flight ahead of the MFMAs that consume them
  auto phase_pv = [&](const bf16x8 (&pf)[4], auto STC) __attribute__((always_inline)) {
    constexpr int ST = decltype(STC)::value;
    constexpr int VIMM = ST * STAGE + TILE_B;
    bf16x8 vf[4][2];
#pragma unroll
    for (int db = 0; db < 2; ++db) vf[0][db] = trans_frag_nw<VIMM>(va[db][0], va[db][1]);
#pragma unroll
    for (int db = 0; db < 2; ++db) vf[1][db] = trans_frag_nw<VIMM + 2048>(va[db][0], va[db][1]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s == 0) {
#pragma unroll
        for (int db = 0; db < 2; ++db) vf[2][db] = trans_frag_nw<VIMM + 2 * 2048>(va[db][0], va[db][1]);
        lgkm_wait<8>(vf[s][0], vf[s][1]);
      } else if (s == 1) {
#pragma unroll
        for (int db = 0; db < 2; ++db) vf[3][db] = trans_frag_nw<VIMM + 3 * 2048>(va[db][0], va[db][1]);
        lgkm_wait<8>(vf[s][0], vf[s][1]);
      } else if (s == 2) {
        lgkm_wait<4>(vf[s][0], vf[s][1]);
      } else {
        lgkm_wait<0>(vf[s][0], vf[s][1]);
      }
#pragma unroll
      for (int db = 0; db < 2; ++db)
        oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[s][db], pf[s], oacc[db], 0, 0, 0);
    }
  };
  // one tile step (ring stage ST: compile-time)
  auto step = [&](int i, auto STC) __attribute__((always_inline)) {
    if (mine - 1 - i >= 1) vm_wait_n<PER_TILE>();  // at most one younger tile in flight
    else vm_wait_n<0>();
    ring_barrier();
    if (i + 2 < mine) issue(i + 2);
    if (i < mine) {
      phase_s(STC);
      bf16x8 pf[4];
      phase_sm(i, pf);
      phase_pv(pf, STC);
    }
  };
  static_assert(S == 3, "the unrolled ring below assumes three stages");
  for (int i = 0; i < per; i += 3) {
    step(i, std::integral_constant<int, 0>{});
    if (i + 1 < per) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < per) step(i + 2, std::integral_constant<int, 2>{});
  }
  vm_wait_n<0>();
  __syncthreads();
  l += __shfl_xor(l, 32, 64);  // the two lane halves of a row hold alternate key groups' sums
  if constexpr (KS > 1) {
    // merge the key-split partials: parts 1.. publish (m, l, O) per lane, part 0 folds them in order
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * QW + wid) * 34 * 64 + lane;
      dst[0] = m;
      dst[64] = l;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(2 + 16 * db + r) * 64] = oacc[db][r];
    }
    __syncthreads();
    if (part > 0) return;
#pragma unroll
    for (int p = 1; p < KS; ++p) {
      const float* src = red + ((p - 1) * QW + wid) * 34 * 64 + lane;
      const float mp = src[0], lp = src[64];
      const float mn = fmaxf(m, mp);
      const float a0 = fast_exp2((m - mn) * LOG2E), a1 = fast_exp2((mp - mn) * LOG2E);
      l = l * a0 + lp * a1;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] = oacc[db][r] * a0 + src[(2 + 16 * db + r) * 64] * a1;
      m = mn;
    }
  }
  const float lsum = l;
  const float inv = 1.0f / lsum;
  if (qok) {
    bf16* orow = o + ((long)n * T + my_q) * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)(oacc[db][4 * g2 + e] * inv);
        *reinterpret_cast<bf16x4*>(orow + 32 * db + 8 * g2 + 4 * hh) = v;
      }
    if (hh == 0) lse[((long)n * heads + h) * T + my_q] = m + logf(lsum);
  }
}


template <int QW, int KS>
__global__ __launch_bounds__(64 * QW * KS) __attribute__((amdgpu_waves_per_eu(2))) void attn_fwd_kernel(
    const bf16* qkv, int ld, int T, int heads, bf16* o, int ldo, float* lse) {
  __shared__ __attribute__((aligned(16))) char smem[FwdLds<QW, KS>::BYTES];
  fwd_segment<QW, KS>(smem, qkv, ld, T, heads, o, ldo, lse, blockIdx.x, blockIdx.y, blockIdx.z, 0, (T + 63) / 64);
}

// ------------------------------------------------------------------------------ backward
// dK/dV: 32 QW keys per block resident in registers (32 per wave); KS query-splits per block (waves
// QW p .. QW p + QW - 1 sweep the p-th range of query tiles), partial dK/dV folded through LDS in a
// fixed order.  Q / dO tiles (+ the rows' -8 lse / -delta) stream through an LDS-DMA ring; Q is not pre-scaled
// (the 1/8 softmax scale is folded into the exp argument and into dK at the end).
//
// Stream-K form (SK, batch-1 shapes whose key-blocks would leave most CUs with one 4-wave block, i.e. one
// wave per SIMD and no MFMA / VALU overlap): G = 2 blocks per CU split the flattened (key-block, query
// tile) space into equal ranges [b U / G, (b + 1) U / G); a block walks its range one key-block segment
// at a time.  A key-block covered by several blocks is finished by the last to arrive: each writes its
// partial dK/dV (sc1 stores, slot b * spb + segment), waits vmcnt(0), and one lane bumps the key-block's
// agent-scope counter; the last arriver reads every covering block's partial back in block order (sc1
// loads), so the sum is independent of arrival order (MI355X_MICROARCH.md hand-off table, row 1), and
// resets the counter.
constexpr int BWD_S = 3;
template <int QW, int KS>
struct DkdvLds {
  static constexpr int STAGE = 2 * TILE_B + 2 * 64 * 4;     // Q, dO, -8 lse, -delta
  static constexpr int RING = KS * BWD_S * STAGE;
  static constexpr int RED = (KS - 1) * QW * 64 * 64 * 4;
  static constexpr int BYTES = RING > RED ? RING : RED;
};

// one key-block (kb, h, n) over query tiles [t0, t0 + tcount); SK: segment `seg` of this block's range
template <int QW, int KS, bool SK>
__device__ __forceinline__ void dkdv_segment(char* smem, const bf16* qkv, int ld, const bf16* dout, int lddo,
                                             const float* nl8, const float* ndel, int T, int heads, bf16* dqkv,
                                             int ldd, int kb, int h, int n, int t0, int tcount, const AttnSK& sk,
                                             long bi, int seg) {
  constexpr int NT = 64 * QW;
  constexpr int S = BWD_S;
  constexpr int STG = DkdvLds<QW, KS>::STAGE;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int part = threadIdx.x / NT, wid = (threadIdx.x >> 6) - part * QW;
  const int lt = threadIdx.x - part * NT;
  char* ring = smem + part * S * STG;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const bf16* dob = dout + (long)n * T * lddo;
  const float* lse_b = nl8 + ((long)n * heads + h) * T;    // -8 lse (raw-score units)
  const float* del_b = ndel + ((long)n * heads + h) * T;   // -delta
  const int my_k = kb * (32 * QW) + wid * 32 + (lane & 31);
  const bool kok = my_k < T;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load_row8(base + (long)my_k * ld + C + h * 64 + 16 * s + 8 * hh, kok, 1.0f);
    vf[s] = load_row8(base + (long)my_k * ld + 2 * C + h * 64 + 16 * s + 8 * hh, kok, 1.0f);
  }
  f32x16 dv[2], dk[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dv[db][r] = 0.0f; dk[db][r] = 0.0f; }

  const int per = (tcount + KS - 1) / KS;
  const int tb = t0 + part * per;
  const int mine = max(0, min(t0 + tcount, tb + per) - tb);
  const __amdgpu_buffer_rsrc_t rq = buf_rsrc(base + h * 64);
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(dob + h * 64);
  const __amdgpu_buffer_rsrc_t rl = buf_rsrc(lse_b);
  const __amdgpu_buffer_rsrc_t rdl = buf_rsrc(del_b);
  TileDma<NT> dq_dma, do_dma;
  dq_dma.init(lt, ld);
  do_dma.init(lt, lddo);
  const int wv = __builtin_amdgcn_readfirstlane(lt >> 6);
  auto issue = [&](int i) __attribute__((always_inline)) {
    char* st = ring + (i % S) * STG;
    const int r0 = (tb + i) * 64;
    dq_dma.issue(rq, st, r0, T, ld, lt);
    do_dma.issue(rd, st + TILE_B, r0, T, lddo, lt);
    if (wv == 0) {  // lse / delta rows of the tile: 64 x 4 B each (rows >= T read 0; their dO rows are 0 too)
      const int soff = __builtin_amdgcn_readfirstlane(r0 * 4);
      buf_load_lds4(rl, (DC_LDS char*)st + 2 * TILE_B, r0 + lane < T ? lane * 4 : kOOB, soff);
      buf_load_lds4(rdl, (DC_LDS char*)st + 2 * TILE_B + 256, r0 + lane < T ? lane * 4 : kOOB, soff);
    }
  };
  // per-lane LDS offsets (loop-invariant)
  int qoff[2][4];
  unsigned ta[2][2][2][2];  // LDS addresses of the transposed pieces (tile + stage offsets are immediates)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
    for (int s = 0; s < 4; ++s) qoff[qb][s] = row_off(32 * qb + (lane & 31), 2 * s + hh);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const TrOff o = tr_off(32 * qb + 16 * s2, 32 * db, lane);
        ta[qb][s2][db][0] = lds_addr(ring) + o.lo;
        ta[qb][s2][db][1] = lds_addr(ring) + o.hi;
      }
  }
  constexpr int PER_TILE = 2 * TileDma<NT>::MIN_INSTR;
  constexpr float L8 = LOG2E * 0.125f;
  for (int i = 0; i < S - 1 && i < mine; ++i) issue(i);
  auto step = [&](int i, auto STC) __attribute__((always_inline)) {
    constexpr int ST = decltype(STC)::value;
    if (mine - 1 - i >= 1) vm_wait_n<PER_TILE>();  // (wave 0 also has the row-constant pieces: conservative)
    else vm_wait_n<0>();
    ring_barrier();
    if (i + S - 1 < mine) issue(i + S - 1);
    if (i < mine) {
      const char* qt_s = ring + ST * STG;
      const char* dt_s = qt_s + TILE_B;
      const float* ls = reinterpret_cast<const float*>(qt_s + 2 * TILE_B);   // -8 lse of the tile's 64 query rows
      const float* dl = ls + 64;                                           // -delta
      // Row constants as the initial accumulators (accumulator element r holds query row
      // 32 qb + 8 (r >> 2) + 4 hh + (r & 3): 4 rows per ds_read_b128): S' = Q K^T - 8 lse and dP' = dO V^T - delta
      // leave the MFMA chains ready for P = exp2(S' log2e / 8) and dS = P dP' -- no per-score subtraction and no
      // per-score lse scaling on the VALU.  Both query halves' S / dP are issued first, so the second half's
      // MFMAs run under the first half's softmax.
      f32x16 spa[2], dpa[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(ls + 32 * qb + 8 * g + 4 * hh);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(dl + 32 * qb + 8 * g + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            spa[qb][4 * g + e] = l4[e];
            dpa[qb][4 * g + e] = d4[e];
          }
        }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          spa[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(qt_s + qoff[qb][s]),
                                                            kf[s], spa[qb], 0, 0, 0);
          dpa[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(dt_s + qoff[qb][s]),
                                                            vf[s], dpa[qb], 0, 0, 0);
        }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x16& sp = spa[qb];
        f32x16& dp = dpa[qb];
        // dO^T / Q^T fragments of the first k-slice, in flight under the softmax
        constexpr int QIMM = ST * STG, DIMM = ST * STG + TILE_B;
        bf16x8 fv[2][2], fk[2][2];
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          fv[0][db] = trans_frag_nw<DIMM>(ta[qb][0][db][0], ta[qb][0][db][1]);
          fk[0][db] = trans_frag_nw<QIMM>(ta[qb][0][db][0], ta[qb][0][db][1]);
        }
        // P = exp2(S' log2e / 8); dS = P dP'
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fast_exp2(sp[r] * L8);
          sp[r] = pv;
          dp[r] *= pv;
        }
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          fv[1][db] = trans_frag_nw<DIMM>(ta[qb][1][db][0], ta[qb][1][db][1]);
          fk[1][db] = trans_frag_nw<QIMM>(ta[qb][1][db][0], ta[qb][1][db][1]);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          if (s2 == 0) lgkm_wait<8>(fv[0][0], fv[0][1], fk[0][0], fk[0][1]);
          else lgkm_wait<0>(fv[1][0], fv[1][1], fk[1][0], fk[1][1]);
          const bf16x8 pf = acc_to_frag(sp, s2);
          const bf16x8 sf = acc_to_frag(dp, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fv[s2][db], pf, dv[db], 0, 0, 0);
            dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fk[s2][db], sf, dk[db], 0, 0, 0);
          }
        }
      }
    }
  };
  static_assert(S == 3, "the unrolled ring below assumes three stages");
  for (int i = 0; i < per; i += 3) {
    step(i, std::integral_constant<int, 0>{});
    if (i + 1 < per) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < per) step(i + 2, std::integral_constant<int, 2>{});
  }
  vm_wait_n<0>();
  __syncthreads();
  if constexpr (KS > 1) {
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * QW + wid) * 64 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dst[(16 * db + r) * 64] = dk[db][r];
          dst[(32 + 16 * db + r) * 64] = dv[db][r];
        }
    }
    __syncthreads();
    if (part > 0) return;
#pragma unroll
    for (int p = 1; p < KS; ++p) {
      const float* src = red + ((p - 1) * QW + wid) * 64 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dk[db][r] += src[(16 * db + r) * 64];
          dv[db][r] += src[(32 + 16 * db + r) * 64];
        }
    }
  }
  if constexpr (SK) {
    const int ntq = (T + 63) / 64;
    if (!(t0 == 0 && tcount == ntq)) {   // key-block shared with other blocks: hand off
      float v[64];
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          v[16 * db + r] = dk[db][r];
          v[32 + 16 * db + r] = dv[db][r];
        }
      if (!sk_handoff<QW, 64>(sk, smem, bi, ntq, seg, v)) return;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dk[db][r] = v[16 * db + r];
          dv[db][r] = v[32 + 16 * db + r];
        }
    }
  }
  if (kok) {
    bf16* row = dqkv + ((long)n * T + my_k) * ldd;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        bf16x4 a, b;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = (bf16)(dk[db][4 * g2 + e] * 0.125f);  // dK = dS^T (Q / 8)
          b[e] = (bf16)dv[db][4 * g2 + e];
        }
        const int d = 32 * db + 8 * g2 + 4 * hh;
        *reinterpret_cast<bf16x4*>(row + C + h * 64 + d) = a;
        *reinterpret_cast<bf16x4*>(row + 2 * C + h * 64 + d) = b;
      }
  }
}

template <int QW, int KS, bool SK>
__global__ __launch_bounds__(64 * QW * KS) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dkdv_kernel(
    const bf16* qkv, int ld, const bf16* dout, int lddo, const float* nl8, const float* ndel, int T, int heads,
    bf16* dqkv, int ldd, AttnSK sk) {
  __shared__ __attribute__((aligned(16))) char smem[DkdvLds<QW, KS>::BYTES];
  const int ntq = (T + 63) / 64;
  if constexpr (!SK) {
    dkdv_segment<QW, KS, false>(smem, qkv, ld, dout, lddo, nl8, ndel, T, heads, dqkv, ldd, blockIdx.x, blockIdx.y,
                                blockIdx.z, 0, ntq, sk, 0, 0);
  } else {
    const int nkb = (T + 32 * QW - 1) / (32 * QW);
    sk_walk(sk, ntq, [&](long bi, int t0, int cnt, int seg) {
      const int kb = (int)(bi % nkb);
      const long nh = bi / nkb;
      dkdv_segment<QW, KS, true>(smem, qkv, ld, dout, lddo, nl8, ndel, T, heads, dqkv, ldd, kb, (int)(nh % heads),
                                 (int)(nh / heads), t0, cnt, sk, bi, seg);
    });
  }
}

// dQ: 32 QW queries per block resident; KS key-splits per block, partial dQ folded through LDS.
// K / V tiles stream through the same LDS-DMA ring as the forward.  Stream-K form as for dK/dV, over
// (query-block, key tile).
template <int QW, int KS>
struct DqLds {
  static constexpr int STAGE = 2 * TILE_B;
  static constexpr int RING = KS * BWD_S * STAGE;
  static constexpr int RED = (KS - 1) * QW * 32 * 64 * 4;
  static constexpr int BYTES = RING > RED ? RING : RED;
};

template <int QW, int KS, bool SK>
__device__ __forceinline__ void dq_segment(char* smem, const bf16* qkv, int ld, const bf16* o, int ldo,
                                           const bf16* dout, int lddo, const float* lse, float* ndel, float* nl8,
                                           int T, int heads, bf16* dqkv, int ldd, int qbk, int h, int n, int t0,
                                           int tcount,
                                           const AttnSK& sk, long bi, int seg) {
  constexpr int NT = 64 * QW;
  constexpr int S = BWD_S;
  constexpr int STG = DqLds<QW, KS>::STAGE;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int part = threadIdx.x / NT, wid = (threadIdx.x >> 6) - part * QW;
  const int lt = threadIdx.x - part * NT;
  char* ring = smem + part * S * STG;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const int my_q = qbk * (32 * QW) + wid * 32 + (lane & 31);
  const bool qok = my_q < T;
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load_row8(base + (long)my_q * ld + h * 64 + 16 * s + 8 * hh, qok, 0.125f);
    df[s] = load_row8(dout + ((long)n * T + my_q) * lddo + h * 64 + 16 * s + 8 * hh, qok, 1.0f);
  }
  const float lse_nat = qok ? lse[((long)n * heads + h) * T + my_q] : INFINITY;
  const float my_lse = lse_nat * LOG2E;
  // delta = sum_d dO * O of this lane's query, from the dO fragments already in registers and the same
  // pieces of O (fp32, fixed order); the key-range segment that starts the row (t0 = 0, part 0) publishes the
  // dK/dV kernel's row constants -delta and -8 lse (it runs after this one)
  float my_del = 0.0f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const bf16x8 of = load_row8(o + ((long)n * T + my_q) * ldo + h * 64 + 16 * s + 8 * hh, qok, 1.0f);
#pragma unroll
    for (int j = 0; j < 8; ++j) my_del = fmaf((float)df[s][j], (float)of[j], my_del);
  }
  my_del += __shfl_xor(my_del, 32, 64);
  if (qok && hh == 0 && part == 0 && t0 == 0) {
    const long r = ((long)n * heads + h) * T + my_q;
    ndel[r] = -my_del;
    nl8[r] = -8.0f * lse_nat;
  }
  f32x16 dq[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[db][r] = 0.0f;
  const int per = (tcount + KS - 1) / KS;
  const int tb = t0 + part * per;
  const int mine = max(0, min(t0 + tcount, tb + per) - tb);
  const __amdgpu_buffer_rsrc_t rk = buf_rsrc(base + C + h * 64);
  const __amdgpu_buffer_rsrc_t rv = buf_rsrc(base + 2 * C + h * 64);
  TileDma<NT> dma;
  dma.init(lt, ld);
  auto issue = [&](int i) __attribute__((always_inline)) {
    char* st = ring + (i % S) * STG;
    dma.issue(rk, st, (tb + i) * 64, T, ld, lt);
    dma.issue(rv, st + TILE_B, (tb + i) * 64, T, ld, lt);
  };
  int koff[2][4];
  unsigned ta[2][2][2][2];  // LDS addresses of the K^T pieces (the stage offset is an immediate)
#pragma unroll
  for (int b = 0; b < 2; ++b) {
#pragma unroll
    for (int s = 0; s < 4; ++s) koff[b][s] = row_off(32 * b + (lane & 31), 2 * s + hh);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const TrOff o = tr_off(32 * b + 16 * s2, 32 * db, lane);
        ta[b][s2][db][0] = lds_addr(ring) + o.lo;
        ta[b][s2][db][1] = lds_addr(ring) + o.hi;
      }
  }
  constexpr int PER_TILE = 2 * TileDma<NT>::MIN_INSTR;
  for (int i = 0; i < S - 1 && i < mine; ++i) issue(i);
  auto step = [&](int i, auto STC) __attribute__((always_inline)) {
    constexpr int ST = decltype(STC)::value;
    if (mine - 1 - i >= 1) vm_wait_n<PER_TILE>();
    else vm_wait_n<0>();
    ring_barrier();
    if (i + S - 1 < mine) issue(i + S - 1);
    if (i < mine) {
      const int kt = tb + i;
      const char* kt_s = ring + ST * STG;
      const char* vt_s = kt_s + TILE_B;
      // S and dP of both key halves first: the second half's MFMAs run under the first half's softmax
      f32x16 spa[2], dpa[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        spa[b] = f32x16{};
        dpa[b] = f32x16{};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          spa[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(kt_s + koff[b][s]), qf[s],
                                                           spa[b], 0, 0, 0);
          dpa[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(vt_s + koff[b][s]), df[s],
                                                           dpa[b], 0, 0, 0);
        }
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x16& sp = spa[b];
        const f32x16& dp = dpa[b];
        // K^T fragments in flight under the softmax
        constexpr int KIMM = ST * STG;
        bf16x8 fq[2][2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int db = 0; db < 2; ++db) fq[s2][db] = trans_frag_nw<KIMM>(ta[b][s2][db][0], ta[b][s2][db][1]);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fast_exp2(fmaf(sp[r], LOG2E, -my_lse));
          sp[r] = pv * (dp[r] - my_del);  // dS^T
        }
        if ((kt + 1) * 64 > T) {  // keys beyond T exist only in the last tile
          asm volatile("" ::: "memory");
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kt * 64 + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * hh >= T) sp[r] = 0.0f;
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          if (s2 == 0) lgkm_wait<4>(fq[0][0], fq[0][1]);
          else lgkm_wait<0>(fq[1][0], fq[1][1]);
          const bf16x8 sf = acc_to_frag(sp, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db)
            dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fq[s2][db], sf, dq[db], 0, 0, 0);
        }
      }
    }
  };
  static_assert(S == 3, "the unrolled ring below assumes three stages");
  for (int i = 0; i < per; i += 3) {
    step(i, std::integral_constant<int, 0>{});
    if (i + 1 < per) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < per) step(i + 2, std::integral_constant<int, 2>{});
  }
  vm_wait_n<0>();
  __syncthreads();
  if constexpr (KS > 1) {
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * QW + wid) * 32 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(16 * db + r) * 64] = dq[db][r];
    }
    __syncthreads();
    if (part > 0) return;
#pragma unroll
    for (int p = 1; p < KS; ++p) {
      const float* src = red + ((p - 1) * QW + wid) * 32 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[db][r] += src[(16 * db + r) * 64];
    }
  }
  if constexpr (SK) {
    const int ntk = (T + 63) / 64;
    if (!(t0 == 0 && tcount == ntk)) {
      float v[32];
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[16 * db + r] = dq[db][r];
      if (!sk_handoff<QW, 32>(sk, smem, bi, ntk, seg, v)) return;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[db][r] = v[16 * db + r];
    }
  }
  if (qok) {
    bf16* row = dqkv + ((long)n * T + my_q) * ldd + h * 64;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        bf16x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = (bf16)(dq[db][4 * g2 + e] * 0.125f);
        *reinterpret_cast<bf16x4*>(row + 32 * db + 8 * g2 + 4 * hh) = a;
      }
  }
}

template <int QW, int KS, bool SK>
__global__ __launch_bounds__(64 * QW * KS) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dq_kernel(
    const bf16* qkv, int ld, const bf16* o, int ldo, const bf16* dout, int lddo, const float* lse, float* ndel,
    float* nl8, int T, int heads, bf16* dqkv, int ldd, AttnSK sk) {
  __shared__ __attribute__((aligned(16))) char smem[DqLds<QW, KS>::BYTES];
  const int ntk = (T + 63) / 64;
  if constexpr (!SK) {
    dq_segment<QW, KS, false>(smem, qkv, ld, o, ldo, dout, lddo, lse, ndel, nl8, T, heads, dqkv, ldd, blockIdx.x,
                              blockIdx.y, blockIdx.z, 0, ntk, sk, 0, 0);
  } else {
    const int nqb = (T + 32 * QW - 1) / (32 * QW);
    sk_walk(sk, ntk, [&](long bi, int t0, int cnt, int seg) {
      const int qbk = (int)(bi % nqb);
      const long nh = bi / nqb;
      dq_segment<QW, KS, true>(smem, qkv, ld, o, ldo, dout, lddo, lse, ndel, nl8, T, heads, dqkv, ldd, qbk,
                               (int)(nh % heads), (int)(nh / heads), t0, cnt, sk, bi, seg);
    });
  }
}


}  // namespace

namespace {
// (query waves per block, key splits per block): chosen per launch by a makespan model over the
// 256 CUs -- rounds of blocks x per-block work (QW) -- discounted when fewer than 8 waves are
// resident per CU.  DC_ATTN_CFG=<index> forces one (tests / benchmarks).
struct AttnCfg {
  int qw, ks, bpc;
};
// (a 6-wave (2, 3) instantiation computed wrong results on gfx950 and is not offered; the others
// are checked one by one in tests/test_gpu_kernels.py::test_attention_fwd_bwd)
constexpr AttnCfg kAttnCfgs[] = {{4, 1, 2}, {4, 2, 1}, {5, 2, 1}, {2, 2, 1}, {4, 3, 1}};
constexpr int kNumAttnCfgs = sizeof(kAttnCfgs) / sizeof(kAttnCfgs[0]);
// the backward kernels hold ~2x the registers: only configs with <= 2 waves per SIMD avoid spills;
// bwd index 2 is (2, 2) (launch_bwd's default case)
constexpr int kNumBwdCfgs = 2;

int attn_cfg(int t, int heads, int nb, bool bwd) {
  const char* e = getenv("DC_ATTN_CFG");  // read per launch (host-side, once per captured graph node)
  const int forced = e ? atoi(e) : -1;
  const int ncfg = bwd ? kNumBwdCfgs : kNumAttnCfgs;
  if (forced >= 0 && forced < (bwd ? kNumBwdCfgs + 1 : kNumAttnCfgs)) return forced;
  // short sequences (levels 2-3 at batch 1: T = 432 / 108, 20 heads): the backward's (2, 2) blocks -- twice the
  // blocks of (4, 2) over the same key tiles -- measured 22.1 vs 26.2 us at T = 432 (profiles/r05aa/); the model
  // below does not see it (it prices resident waves, not the sequential key-tile chain of a small grid)
  if (bwd && (long)t * nb <= 512) return 2;
  // many blocks (batch 8 / the C5 ensemble): the forward's (4, 1) -- three 4-wave blocks per CU -- beats the 10-wave
  // key-split blocks the model below prefers (L0 batch 8 605 vs 653 us, L2 batch 8 23.9 vs 26.3 us; batch 1, where
  // (4, 1) leaves one block per CU, keeps (5, 2): 104 vs 142 us; profiles/r06d/)
  if (!bwd && (long)((t + 127) / 128) * heads * nb > 2L * 256) return 0;
  int best = 0;
  double best_t = 1e30;
  for (int i = 0; i < ncfg; ++i) {
    const AttnCfg c = kAttnCfgs[i];
    const long blocks = (long)((t + 32 * c.qw - 1) / (32 * c.qw)) * heads * nb;
    const long per_cu = (blocks + 255) / 256;
    const long resident = (long)c.qw * c.ks * (per_cu < c.bpc ? per_cu : c.bpc);
    const double eff = resident >= 8 ? 1.0 : resident / 8.0;
    const double tm = (double)per_cu * c.qw / eff;
    if (tm < best_t * 0.999) { best_t = tm; best = i; }
  }
  return best;
}

template <int QW, int KS>
void launch_fwd(const bf16* qkv, int ld, int t, int heads, int nb, bf16* o, int ldo, float* lse, hipStream_t st) {
  dim3 grid((t + 32 * QW - 1) / (32 * QW), heads, nb);
  hipLaunchKernelGGL((attn_fwd_kernel<QW, KS>), grid, dim3(64 * QW * KS), 0, st, qkv, ld, t, heads, o, ldo, lse);
}

// dQ first: it computes delta = rowsum(dO * O) for its resident queries and publishes the dK/dV kernel's row
// constants -delta (delta[0, nht)) and -8 lse (delta[nht, 2 nht)); dK/dV (next launch, same stream) reads them --
// no separate delta pass
template <int QW, int KS>
void launch_bwd(const bf16* qkv, int ld, const bf16* o, int ldo, const bf16* dout, int lddo, const float* lse,
                float* delta, int t, int heads, int nb, bf16* dqkv, int ldd, bool with_dq, bool with_dkdv,
                hipStream_t st) {
  dim3 grid((t + 32 * QW - 1) / (32 * QW), heads, nb);
  const AttnSK none{};
  float* nl8 = delta + (long)nb * heads * t;
  if (with_dq)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<QW, KS, false>), grid, dim3(64 * QW * KS), 0, st, qkv, ld, o, ldo, dout,
                       lddo, lse, delta, nl8, t, heads, dqkv, ldd, none);
  if (with_dkdv)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<QW, KS, false>), grid, dim3(64 * QW * KS), 0, st, qkv, ld, dout, lddo,
                       nl8, delta, t, heads, dqkv, ldd, none);
}

int device_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return cus[dev];
}

// Stream-K backward (4-wave blocks, 2 per CU) when the plain grid would leave CUs with a single 4-wave
// block; the partial slab lives in ws, the per-block counters in its last 64 KB (shared with
// dc_conv_gemm's, all self-resetting).  DC_ATTN_SK=0 disables it.  Returns false when it does not apply.
constexpr long kAttnCounterBytes = 64 * 1024;
// stream-K plan for QW = 4 blocks (2 per CU): false when it does not apply; `env` names the switch
bool sk_plan(int t, int heads, int nb, float* ws, long ws_bytes, const char* env_name, AttnSK& sk) {
  constexpr int QW = 4;
  const char* env = getenv(env_name);   // read per launch (host side, once per captured graph node)
  if (!ws || (env && atoi(env) == 0)) return false;
  const long units_blocks = (long)((t + 32 * QW - 1) / (32 * QW)) * heads * nb;
  const int ntile = (t + 63) / 64;
  const long G = 2L * device_cus();
  const long U = units_blocks * ntile;
  const bool forced = env && atoi(env) == 2;   // tests: take the stream-K form wherever it fits
  // per-segment costs (K/V registers, ring prologue, partial hand-off) need >= 32 tiles per block to
  // amortise: UNet level 0 at batch 1 (57 per block) gains 19 %, level 1 (7 per block) loses 30 %
  if (!forced && (units_blocks >= G || U < 32 * G)) return false;
  if (units_blocks > kAttnCounterBytes / 4 || U < 2) return false;
  const long g = min(G, U);
  const int spb = (int)(((U + g - 1) / g + ntile - 1) / ntile + 1);
  if (g * spb * QW * 64L * 64 * 4 > ws_bytes - kAttnCounterBytes) return false;
  sk.slab = ws;
  sk.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(ws) + (ws_bytes - kAttnCounterBytes));
  sk.U = U;
  sk.G = (int)g;
  sk.spb = spb;
  return true;
}

bool launch_bwd_sk(const bf16* qkv, int ld, const bf16* o, int ldo, const bf16* dout, int lddo, const float* lse,
                   float* delta, int t, int heads, int nb, bf16* dqkv, int ldd, float* ws, long ws_bytes,
                   bool with_dq, bool with_dkdv, hipStream_t st) {
  AttnSK sk;
  if (!sk_plan(t, heads, nb, ws, ws_bytes, "DC_ATTN_SK", sk)) return false;
  float* nl8 = delta + (long)nb * heads * t;
  if (with_dq)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<4, 1, true>), dim3((unsigned)sk.G), dim3(256), 0, st, qkv, ld, o, ldo, dout,
                       lddo, lse, delta, nl8, t, heads, dqkv, ldd, sk);
  if (with_dkdv)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<4, 1, true>), dim3((unsigned)sk.G), dim3(256), 0, st, qkv, ld, dout,
                       lddo, nl8, delta, t, heads, dqkv, ldd, sk);
  return true;
}

}  // namespace

extern "C" int dc_attn_fwd(const void* qkv, int ld, int nb, int t, int heads, void* o, int ldo, float* lse,
                           float* ws, long long ws_bytes, void* stream) {
  if (!qkv || !o || !lse || nb <= 0 || t <= 0 || heads <= 0) return DC_ERR_ARG;
  if (ld % 8 || ldo % 8 || ld < 3 * heads * 64 || ldo < heads * 64) return DC_ERR_ALIGN;
  const bf16* q = (const bf16*)qkv;
  hipStream_t st = (hipStream_t)stream;
  (void)ws;
  (void)ws_bytes;
  switch (attn_cfg(t, heads, nb, false)) {
    case 0: launch_fwd<4, 1>(q, ld, t, heads, nb, (bf16*)o, ldo, lse, st); break;
    case 1: launch_fwd<4, 2>(q, ld, t, heads, nb, (bf16*)o, ldo, lse, st); break;
    case 2: launch_fwd<5, 2>(q, ld, t, heads, nb, (bf16*)o, ldo, lse, st); break;
    case 3: launch_fwd<2, 2>(q, ld, t, heads, nb, (bf16*)o, ldo, lse, st); break;
    default: launch_fwd<4, 3>(q, ld, t, heads, nb, (bf16*)o, ldo, lse, st); break;
  }
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_attn_bwd(const void* qkv, int ld, const void* o, int ldo, const void* dout, int lddo,
                           const float* lse, int nb, int t, int heads, float* delta_ws, void* dqkv, int ldd,
                           float* ws, long long ws_bytes, void* stream) {
  if (!qkv || !o || !dout || !lse || !delta_ws || !dqkv || nb <= 0 || t <= 0 || heads <= 0) return DC_ERR_ARG;
  if (ld % 8 || ldo % 8 || lddo % 8 || ldd % 8 || ldd < 3 * heads * 64) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const bf16* q = (const bf16*)qkv;
  const bf16* ob = (const bf16*)o;
  const bf16* d = (const bf16*)dout;
  bf16* g = (bf16*)dqkv;
  const long wsb = ws_bytes < (1LL << 40) ? (long)ws_bytes : 0;
  // dQ first (it publishes the row constants for dK/dV), then dK/dV: by the stream-K kernels where the plan applies, else on
  // the plain grid
  if (!launch_bwd_sk(q, ld, ob, ldo, d, lddo, lse, delta_ws, t, heads, nb, g, ldd, ws, wsb, true, true, st)) {
    const int cfg = attn_cfg(t, heads, nb, true);
    if (cfg == 0)
      launch_bwd<4, 1>(q, ld, ob, ldo, d, lddo, lse, delta_ws, t, heads, nb, g, ldd, true, true, st);
    else if (cfg == 1)
      launch_bwd<4, 2>(q, ld, ob, ldo, d, lddo, lse, delta_ws, t, heads, nb, g, ldd, true, true, st);
    else
      launch_bwd<2, 2>(q, ld, ob, ldo, d, lddo, lse, delta_ws, t, heads, nb, g, ldd, true, true, st);
  }
  DC_CHECK_LAUNCH();
  return DC_OK;
}
