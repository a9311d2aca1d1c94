// Self-attention (flash-style, head dim 64) forward / backward and the folded 2-key
// cross-attention of the UNet's Transformer2DModel blocks (gfx950, MFMA 32x32x16 bf16).
//
// Layouts: qkv [nb*T][ld] bf16 with q | k | v column blocks (head h at column h*64 of each block),
// o [nb*T][ldo], lse [nb][heads][T] fp32 (natural log of sum exp(q.k/8)).
// The forward keeps S^T = K Q^T in registers (query on the lane), so softmax row statistics are
// lane-local; P feeds the P.V MFMA straight from the accumulator (O^T = V^T P^T) with V^T fragments
// from ds_read_b64_tr_b16.  The backward is split into a dK/dV kernel (keys resident per wave,
// sweeping queries) and a dQ kernel (queries resident, sweeping keys): deterministic, no atomics.
#include "common.h"
#include "../../include/dcamd.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
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

// stage a [64 rows][64 cols] bf16 tile (rows r0.., column offset col) into LDS with `stride`
__device__ __forceinline__ void stage_load(const bf16* base, long ld, int r0, int rows_total, int col, uint4 (&reg)[2],
                                           int t) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i, piece = t & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < rows_total) v = *reinterpret_cast<const uint4*>(base + (long)(r0 + row) * ld + col + piece * 8);
    reg[i] = v;
  }
}
__device__ __forceinline__ void stage_store(bf16* tile, int stride, const uint4 (&reg)[2], float scale, int t) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i, piece = t & 7;
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

// ------------------------------------------------------------------------------ forward
// KS key-splits per block: waves 4p..4p+3 sweep the p-th contiguous range of key tiles for the same
// 128 queries (KS x 4 waves per CU hide MFMA / softmax / LDS latency at small T x heads), then the
// partial (m, l, O) are merged through LDS in a fixed order (deterministic).
template <int KS>
struct FwdLds {
  static constexpr int K_BYTES = KS * 2 * 64 * KSTR * 2;
  static constexpr int V_BYTES = KS * 2 * 64 * VSTR * 2;
  static constexpr int RED = (KS - 1) * 4 * 34 * 64 * 4;
  static constexpr int BYTES = (K_BYTES + V_BYTES > RED) ? K_BYTES + V_BYTES : RED;
};

template <int KS>
__global__ __launch_bounds__(256 * KS) void attn_fwd_kernel(const bf16* qkv, int ld, int T, int heads, bf16* o,
                                                            int ldo, float* lse) {
  __shared__ __attribute__((aligned(16))) char smem[FwdLds<KS>::BYTES];
  const int lane = threadIdx.x & 63, wid = (threadIdx.x >> 6) & 3, part = threadIdx.x >> 8, hh = lane >> 5;
  const int lt = threadIdx.x & 255;
  bf16* ks = reinterpret_cast<bf16*>(smem) + part * 2 * 64 * KSTR;
  bf16* vs = reinterpret_cast<bf16*>(smem + FwdLds<KS>::K_BYTES) + part * 2 * 64 * VSTR;
  const int h = blockIdx.y, n = blockIdx.z;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const int my_q = blockIdx.x * 128 + wid * 32 + (lane & 31);
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

  const int ntiles = (T + 63) / 64;
  const int per = (ntiles + KS - 1) / KS;
  const int tb = part * per;
  const int mine = max(0, min(ntiles, tb + per) - tb);
  uint4 rk[2], rv[2];
  if (mine > 0) {
    stage_load(base, ld, tb * 64, T, C + h * 64, rk, lt);
    stage_load(base, ld, tb * 64, T, 2 * C + h * 64, rv, lt);
    stage_store(ks, KSTR, rk, 1.0f, lt);
    stage_store(vs, VSTR, rv, 1.0f, lt);
  }
  __syncthreads();
  for (int i = 0; i < per; ++i) {
    const int kt = tb + i;
    const int cur = i & 1;
    const bool more = i + 1 < mine;
    if (more) {
      stage_load(base, ld, (kt + 1) * 64, T, C + h * 64, rk, lt);
      stage_load(base, ld, (kt + 1) * 64, T, 2 * C + h * 64, rv, lt);
    }
    if (i < mine) {
      const bf16* kt_s = ks + cur * 64 * KSTR;
      const bf16* vt_s = vs + cur * 64 * VSTR;
      f32x16 sacc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[b][r] = 0.0f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt_s + (32 * b + (lane & 31)) * KSTR + 16 * s + 8 * hh);
          sacc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[b], 0, 0, 0);
        }
      }
      // scores -> log2 domain, mask keys beyond T
      float mx = -INFINITY;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 64 + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * hh;
          float v = sacc[b][r] * LOG2E;
          v = key < T ? v : -INFINITY;
          sacc[b][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float alpha = exp2f(m - mnew);
      float ps = 0.0f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = exp2f(sacc[b][r] - mnew);
          sacc[b][r] = pv;
          ps += pv;
        }
      l = l * alpha + ps;
      m = mnew;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] *= alpha;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 pf = acc_to_frag(sacc[s >> 1], s & 1);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const bf16x8 vf = trans_frag(vt_s, VSTR, 16 * s, 32 * db, lane);
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[db], 0, 0, 0);
        }
      }
    }
    if (more) {
      stage_store(ks + (cur ^ 1) * 64 * KSTR, KSTR, rk, 1.0f, lt);
      stage_store(vs + (cur ^ 1) * 64 * VSTR, VSTR, rv, 1.0f, lt);
    }
    __syncthreads();
  }
  if constexpr (KS > 1) {
    // merge the key-split partials: parts 1.. publish (m, l, O) per lane, part 0 folds them in order
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * 4 + wid) * 34 * 64 + lane;
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
      const float* src = red + ((p - 1) * 4 + wid) * 34 * 64 + lane;
      const float mp = src[0], lp = src[64];
      const float mn = fmaxf(m, mp);
      const float a0 = exp2f(m - mn), a1 = exp2f(mp - mn);
      l = l * a0 + lp * a1;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] = oacc[db][r] * a0 + src[(2 + 16 * db + r) * 64] * a1;
      m = mn;
    }
  }
  const float lsum = l + __shfl_xor(l, 32, 64);
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
    if (hh == 0) lse[((long)n * heads + h) * T + my_q] = m * LN2 + logf(lsum);
  }
}

// ------------------------------------------------------------------------------ backward
// delta[n][h][q] = sum_d dO * O  (fp32)
__global__ void attn_delta_kernel(const bf16* o, int ldo, const bf16* dout, int lddo, int T, int heads, long total,
                                  float* delta) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int h = (int)(idx % heads);
  const long nq = idx / heads;  // n*T + q
  const int q = (int)(nq % T);
  const long n = nq / T;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a[8], b[8];
    load8(o + nq * ldo + h * 64 + 8 * k, a);
    load8(dout + nq * lddo + h * 64 + 8 * k, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * b[i];
  }
  delta[(n * heads + h) * T + q] = s;
}

// dK/dV: 128 keys per block resident in registers (32 per wave); KS query-splits per block (waves
// 4p..4p+3 sweep the p-th range of query tiles), partial dK/dV folded through LDS in a fixed order.
template <int KS>
struct DkdvLds {
  static constexpr int TILE = 64 * KSTR * 2;
  static constexpr int MAIN = KS * 2 * 2 * TILE + KS * 2 * 2 * 64 * 4;
  static constexpr int RED = (KS - 1) * 4 * 64 * 64 * 4;
  static constexpr int BYTES = MAIN > RED ? MAIN : RED;
};

template <int KS>
__global__ __launch_bounds__(256 * KS) void attn_bwd_dkdv_kernel(const bf16* qkv, int ld, const bf16* dout, int lddo,
                                                                 const float* lse, const float* delta, int T,
                                                                 int heads, bf16* dqkv, int ldd) {
  __shared__ __attribute__((aligned(16))) char smem[DkdvLds<KS>::BYTES];
  const int lane = threadIdx.x & 63, wid = (threadIdx.x >> 6) & 3, part = threadIdx.x >> 8, hh = lane >> 5;
  const int lt = threadIdx.x & 255;
  constexpr int TILE = DkdvLds<KS>::TILE;
  bf16* qs = reinterpret_cast<bf16*>(smem + part * 2 * 2 * TILE);       // [2 stages][64 * KSTR]
  bf16* ds_ = reinterpret_cast<bf16*>(smem + part * 2 * 2 * TILE + 2 * TILE);
  float* ls = reinterpret_cast<float*>(smem + KS * 2 * 2 * TILE) + part * 2 * 2 * 64;  // [2][64]
  float* dl = ls + 2 * 64;
  const int h = blockIdx.y, n = blockIdx.z;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const bf16* dob = dout + (long)n * T * lddo;
  const float* lse_b = lse + ((long)n * heads + h) * T;
  const float* del_b = delta + ((long)n * heads + h) * T;
  const int my_k = blockIdx.x * 128 + wid * 32 + (lane & 31);
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

  const int ntiles = (T + 63) / 64;
  const int per = (ntiles + KS - 1) / KS;
  const int tb = part * per;
  const int mine = max(0, min(ntiles, tb + per) - tb);
  uint4 rq[2], rd[2];
  float rl = 0.0f, rdl = 0.0f;
  auto load_tile = [&](int qt) {
    stage_load(base, ld, qt * 64, T, h * 64, rq, lt);
    stage_load(dob, lddo, qt * 64, T, h * 64, rd, lt);
    if (lt < 64) {
      const int q = qt * 64 + lt;
      rl = q < T ? lse_b[q] : INFINITY;
      rdl = q < T ? del_b[q] : 0.0f;
    }
  };
  auto store_tile = [&](int st) {
    stage_store(qs + st * 64 * KSTR, KSTR, rq, 0.125f, lt);
    stage_store(ds_ + st * 64 * KSTR, KSTR, rd, 1.0f, lt);
    if (lt < 64) {
      ls[st * 64 + lt] = rl;
      dl[st * 64 + lt] = rdl;
    }
  };
  if (mine > 0) {
    load_tile(tb);
    store_tile(0);
  }
  __syncthreads();
  for (int i = 0; i < per; ++i) {
    const int qt = tb + i;
    const int cur = i & 1;
    const bool more = i + 1 < mine;
    if (more) load_tile(qt + 1);
    if (i < mine) {
      const bf16* qt_s = qs + cur * 64 * KSTR;
      const bf16* dt_s = ds_ + cur * 64 * KSTR;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x16 sp, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = 32 * qb + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sp[r] = -ls[cur * 64 + qr];
          dp[r] = -dl[cur * 64 + qr];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 qa =
              *reinterpret_cast<const bf16x8*>(qt_s + (32 * qb + (lane & 31)) * KSTR + 16 * s + 8 * hh);
          sp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], sp, 0, 0, 0);
          const bf16x8 da =
              *reinterpret_cast<const bf16x8*>(dt_s + (32 * qb + (lane & 31)) * KSTR + 16 * s + 8 * hh);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[s], dp, 0, 0, 0);
        }
        // sp = S - lse -> P ; dp = dP - delta -> dS = P * dp
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = exp2f(sp[r] * LOG2E);
          sp[r] = pv;
          dp[r] = pv * dp[r];
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pf = acc_to_frag(sp, s2);
          const bf16x8 sf = acc_to_frag(dp, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const bf16x8 doT = trans_frag(dt_s, KSTR, 32 * qb + 16 * s2, 32 * db, lane);
            dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(doT, pf, dv[db], 0, 0, 0);
            const bf16x8 qT = trans_frag(qt_s, KSTR, 32 * qb + 16 * s2, 32 * db, lane);
            dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qT, sf, dk[db], 0, 0, 0);
          }
        }
      }
    }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }
  if constexpr (KS > 1) {
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * 4 + wid) * 64 * 64 + lane;
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
      const float* src = red + ((p - 1) * 4 + wid) * 64 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dk[db][r] += src[(16 * db + r) * 64];
          dv[db][r] += src[(32 + 16 * db + r) * 64];
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
          a[e] = (bf16)dk[db][4 * g2 + e];
          b[e] = (bf16)dv[db][4 * g2 + e];
        }
        const int d = 32 * db + 8 * g2 + 4 * hh;
        *reinterpret_cast<bf16x4*>(row + C + h * 64 + d) = a;
        *reinterpret_cast<bf16x4*>(row + 2 * C + h * 64 + d) = b;
      }
  }
}

// dQ: 128 queries per block resident; KS key-splits per block, partial dQ folded through LDS.
template <int KS>
struct DqLds {
  static constexpr int TILE = 64 * KSTR * 2;
  static constexpr int MAIN = KS * 2 * 2 * TILE;
  static constexpr int RED = (KS - 1) * 4 * 32 * 64 * 4;
  static constexpr int BYTES = MAIN > RED ? MAIN : RED;
};

template <int KS>
__global__ __launch_bounds__(256 * KS) void attn_bwd_dq_kernel(const bf16* qkv, int ld, const bf16* dout, int lddo,
                                                               const float* lse, const float* delta, int T, int heads,
                                                               bf16* dqkv, int ldd) {
  __shared__ __attribute__((aligned(16))) char smem[DqLds<KS>::BYTES];
  const int lane = threadIdx.x & 63, wid = (threadIdx.x >> 6) & 3, part = threadIdx.x >> 8, hh = lane >> 5;
  const int lt = threadIdx.x & 255;
  constexpr int TILE = DqLds<KS>::TILE;
  bf16* ks = reinterpret_cast<bf16*>(smem + part * 2 * 2 * TILE);
  bf16* vs = reinterpret_cast<bf16*>(smem + part * 2 * 2 * TILE + 2 * TILE);
  const int h = blockIdx.y, n = blockIdx.z;
  const int C = heads * 64;
  const bf16* base = qkv + (long)n * T * ld;
  const int my_q = blockIdx.x * 128 + wid * 32 + (lane & 31);
  const bool qok = my_q < T;
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load_row8(base + (long)my_q * ld + h * 64 + 16 * s + 8 * hh, qok, 0.125f);
    df[s] = load_row8(dout + ((long)n * T + my_q) * lddo + h * 64 + 16 * s + 8 * hh, qok, 1.0f);
  }
  const float my_lse = qok ? lse[((long)n * heads + h) * T + my_q] * LOG2E : INFINITY;
  const float my_del = qok ? delta[((long)n * heads + h) * T + my_q] : 0.0f;
  f32x16 dq[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[db][r] = 0.0f;
  const int ntiles = (T + 63) / 64;
  const int per = (ntiles + KS - 1) / KS;
  const int tb = part * per;
  const int mine = max(0, min(ntiles, tb + per) - tb);
  uint4 rk[2], rv[2];
  if (mine > 0) {
    stage_load(base, ld, tb * 64, T, C + h * 64, rk, lt);
    stage_load(base, ld, tb * 64, T, 2 * C + h * 64, rv, lt);
    stage_store(ks, KSTR, rk, 1.0f, lt);
    stage_store(vs, KSTR, rv, 1.0f, lt);
  }
  __syncthreads();
  for (int i = 0; i < per; ++i) {
    const int kt = tb + i;
    const int cur = i & 1;
    const bool more = i + 1 < mine;
    if (more) {
      stage_load(base, ld, (kt + 1) * 64, T, C + h * 64, rk, lt);
      stage_load(base, ld, (kt + 1) * 64, T, 2 * C + h * 64, rv, lt);
    }
    if (i < mine) {
      const bf16* kt_s = ks + cur * 64 * KSTR;
      const bf16* vt_s = vs + cur * 64 * KSTR;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x16 sp, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { sp[r] = 0.0f; dp[r] = 0.0f; }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 ka = *reinterpret_cast<const bf16x8*>(kt_s + (32 * b + (lane & 31)) * KSTR + 16 * s + 8 * hh);
          sp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sp, 0, 0, 0);
          const bf16x8 va = *reinterpret_cast<const bf16x8*>(vt_s + (32 * b + (lane & 31)) * KSTR + 16 * s + 8 * hh);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, df[s], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 64 + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const float pv = key < T ? exp2f(sp[r] * LOG2E - my_lse) : 0.0f;
          sp[r] = pv * (dp[r] - my_del);  // dS^T
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 sf = acc_to_frag(sp, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const bf16x8 kT = trans_frag(kt_s, KSTR, 32 * b + 16 * s2, 32 * db, lane);
            dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kT, sf, dq[db], 0, 0, 0);
          }
        }
      }
    }
    if (more) {
      stage_store(ks + (cur ^ 1) * 64 * KSTR, KSTR, rk, 1.0f, lt);
      stage_store(vs + (cur ^ 1) * 64 * KSTR, KSTR, rv, 1.0f, lt);
    }
    __syncthreads();
  }
  if constexpr (KS > 1) {
    float* red = reinterpret_cast<float*>(smem);
    if (part > 0) {
      float* dst = red + ((part - 1) * 4 + wid) * 32 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(16 * db + r) * 64] = dq[db][r];
    }
    __syncthreads();
    if (part > 0) return;
#pragma unroll
    for (int p = 1; p < KS; ++p) {
      const float* src = red + ((p - 1) * 4 + wid) * 32 * 64 + lane;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[db][r] += src[(16 * db + r) * 64];
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

// ------------------------------------------------------------------ folded 2-key cross-attention
// attn2(LN2(x)) with a constant 2-token context reduces exactly to
//   out = x + c0 + sum_h sigmoid(LN2(x) . U_h) * D_h        (U, D: [H][C] fp32, c0: [C] fp32)
// (U_h = Wq_h^T (k1_h - k2_h)/8, D_h = Wo_h (v1_h - v2_h), c0 = Wo v2 + bo).
template <int MAXV>
__global__ void cross_fwd_kernel(const bf16* x, int ldx, long rows, int c, int heads, float eps, const float* gamma,
                                 const float* beta, const float* U, const float* D, const float* c0, bf16* y, int ldy,
                                 float* stats, float* probs) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  float xv[MAXV][8], nn[MAXV][8];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      load8(x + row * ldx + vi * 8, xv[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += xv[k][i];
    }
  }
  const float mu = wave_sum(s) / c;
  float q = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = xv[k][i] - mu; q += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(q) / c + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        nn[k][i] = (float)(bf16)((xv[k][i] - mu) * rs * gamma[vi * 8 + i] + beta[vi * 8 + i]);
    }
  }
  float acc[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[k][i] = 0.0f;
  for (int hd = 0; hd < heads; ++hd) {
    float d = 0.0f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nv) {
#pragma unroll
        for (int i = 0; i < 8; ++i) d += nn[k][i] * U[(long)hd * c + vi * 8 + i];
      }
    }
    d = wave_sum(d);
    const float p = 1.0f / (1.0f + __expf(-d));
    if (lane == 0) probs[row * heads + hd] = p;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nv) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[k][i] += p * D[(long)hd * c + vi * 8 + i];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)(acc[k][i] + c0[vi * 8 + i]) + xv[k][i];
      store8(y + row * ldy + vi * 8, o);
    }
  }
  if (lane == 0) {
    stats[row * 2] = mu;
    stats[row * 2 + 1] = rs;
  }
}

template <int MAXV>
__global__ void cross_bwd_kernel(const bf16* x, int ldx, long rows, int c, int heads, const float* gamma,
                                 const float* U, const float* D, const float* stats, const float* probs,
                                 const bf16* dy, int lddy, bf16* dx, int lddx) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  float dv[MAXV][8], dn[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
#pragma unroll
    for (int i = 0; i < 8; ++i) dn[k][i] = 0.0f;
    if (vi < nv) load8(dy + row * lddy + vi * 8, dv[k]);
  }
  for (int hd = 0; hd < heads; ++hd) {
    float d = 0.0f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nv) {
#pragma unroll
        for (int i = 0; i < 8; ++i) d += dv[k][i] * D[(long)hd * c + vi * 8 + i];
      }
    }
    d = wave_sum(d);
    const float p = probs[row * heads + hd];
    const float dsg = d * p * (1.0f - p);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nv) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dn[k][i] += dsg * U[(long)hd * c + vi * 8 + i];
      }
    }
  }
  // LayerNorm backward of dn, plus the residual path
  const float mu = stats[row * 2], rs = stats[row * 2 + 1];
  float xh[MAXV][8];
  float sa = 0.0f, sb = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float f[8];
      load8(x + row * ldx + vi * 8, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[k][i] = (f[i] - mu) * rs;
        dn[k][i] = (float)(bf16)dn[k][i] * gamma[vi * 8 + i];
        sa += dn[k][i];
        sb += dn[k][i] * xh[k][i];
      }
    }
  }
  const float ma = wave_sum(sa) / c, mb = wave_sum(sb) / c;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)(rs * (dn[k][i] - ma - xh[k][i] * mb)) + dv[k][i];
      store8(dx + row * lddx + vi * 8, o);
    }
  }
}

}  // namespace

namespace {
// DC_ATTN_KS=1|2 overrides the automatic choice (benchmarks / tests)
int attn_ks(dim3 grid) {
  static int forced = [] {
    const char* e = getenv("DC_ATTN_KS");
    return e ? atoi(e) : 0;
  }();
  if (forced == 1 || forced == 2) return forced;
  return (long)grid.x * grid.y * grid.z < 1024 ? 2 : 1;
}
}  // namespace

extern "C" int dc_attn_fwd(const void* qkv, int ld, int nb, int t, int heads, void* o, int ldo, float* lse,
                           void* stream) {
  if (!qkv || !o || !lse || nb <= 0 || t <= 0 || heads <= 0) return DC_ERR_ARG;
  if (ld % 8 || ldo % 8 || ld < 3 * heads * 64 || ldo < heads * 64) return DC_ERR_ALIGN;
  dim3 grid((t + 127) / 128, heads, nb);
  // key-split factor: enough resident waves per CU when (query blocks x heads x frames) is small
  if (attn_ks(grid) == 2)
    hipLaunchKernelGGL(attn_fwd_kernel<2>, grid, dim3(512), 0, (hipStream_t)stream, (const bf16*)qkv, ld, t, heads,
                       (bf16*)o, ldo, lse);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)qkv, ld, t, heads,
                       (bf16*)o, ldo, lse);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_attn_bwd(const void* qkv, int ld, const void* o, int ldo, const void* dout, int lddo,
                           const float* lse, int nb, int t, int heads, float* delta_ws, void* dqkv, int ldd,
                           void* stream) {
  if (!qkv || !o || !dout || !lse || !delta_ws || !dqkv || nb <= 0 || t <= 0 || heads <= 0) return DC_ERR_ARG;
  if (ld % 8 || ldo % 8 || lddo % 8 || ldd % 8 || ldd < 3 * heads * 64) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const long total = (long)nb * t * heads;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const bf16*)o, ldo,
                     (const bf16*)dout, lddo, t, heads, total, delta_ws);
  dim3 grid((t + 127) / 128, heads, nb);
  if (attn_ks(grid) == 2) {
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<2>, grid, dim3(512), 0, st, (const bf16*)qkv, ld, (const bf16*)dout, lddo,
                       lse, delta_ws, t, heads, (bf16*)dqkv, ldd);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<2>, grid, dim3(512), 0, st, (const bf16*)qkv, ld, (const bf16*)dout, lddo,
                       lse, delta_ws, t, heads, (bf16*)dqkv, ldd);
  } else {
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<1>, grid, dim3(256), 0, st, (const bf16*)qkv, ld, (const bf16*)dout, lddo,
                       lse, delta_ws, t, heads, (bf16*)dqkv, ldd);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<1>, grid, dim3(256), 0, st, (const bf16*)qkv, ld, (const bf16*)dout, lddo,
                       lse, delta_ws, t, heads, (bf16*)dqkv, ldd);
  }
  DC_CHECK_LAUNCH();
  return DC_OK;
}

#define DC_CROSS_DISPATCH(KER, ...)                                                            \
  do {                                                                                         \
    const int nv = c / 8;                                                                      \
    dim3 grid((unsigned)((rows + 3) / 4));                                                     \
    if (nv <= 64)                                                                              \
      hipLaunchKernelGGL(KER<1>, grid, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__);        \
    else if (nv <= 192)                                                                        \
      hipLaunchKernelGGL(KER<3>, grid, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__);        \
    else if (nv <= 320)                                                                        \
      hipLaunchKernelGGL(KER<5>, grid, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__);        \
    else                                                                                       \
      return DC_ERR_ARG;                                                                       \
  } while (0)

extern "C" int dc_crossattn_fwd(const void* x, int ldx, long long rows, int c, int heads, float eps,
                                const float* gamma, const float* beta, const float* U, const float* D,
                                const float* c0, void* y, int ldy, float* stats, float* probs, void* stream) {
  if (!x || !y || !gamma || !beta || !U || !D || !c0 || !stats || !probs || rows <= 0 || c % 8 || heads <= 0)
    return DC_ERR_ARG;
  if (ldx % 8 || ldy % 8) return DC_ERR_ALIGN;
  DC_CROSS_DISPATCH(cross_fwd_kernel, (const bf16*)x, ldx, (long)rows, c, heads, eps, gamma, beta, U, D, c0, (bf16*)y,
                    ldy, stats, probs);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_crossattn_bwd(const void* x, int ldx, long long rows, int c, int heads, const float* gamma,
                                const float* U, const float* D, const float* stats, const float* probs,
                                const void* dy, int lddy, void* dx, int lddx, void* stream) {
  if (!x || !dy || !dx || !gamma || !U || !D || !stats || !probs || rows <= 0 || c % 8 || heads <= 0)
    return DC_ERR_ARG;
  if (ldx % 8 || lddy % 8 || lddx % 8) return DC_ERR_ALIGN;
  DC_CROSS_DISPATCH(cross_bwd_kernel, (const bf16*)x, ldx, (long)rows, c, heads, gamma, U, D, stats, probs,
                    (const bf16*)dy, lddy, (bf16*)dx, lddx);
  DC_CHECK_LAUNCH();
  return DC_OK;
}
