// Implicit-GEMM convolution / linear layer on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
// One kernel serves every matmul-shaped op of the hot path:
//   * 3x3 / 1x1 convs of the UNet resnets and TAESD (fwd), stride 2 (Downsample2D),
//     nearest-upsample folded into the A-operand addressing (Upsample2D, TAESD Upsample),
//   * their input gradients (dgrad = conv with pre-flipped/transposed weights; mode 2 is
//     the transposed stride-2 gather for the Downsample2D VJP),
//   * every nn.Linear (1x1 conv over token rows).
// GEMM view: M = output pixels (NHWC rows), N = output channels, K = taps x Cin (K contiguous
// in both operands).  Tiles: BM x BN x 64, 4 waves (2x2), register-staged double-buffered LDS
// with an XOR swizzle (conflict-free ds_read_b128 fragments), LDS-staged coalesced epilogue
// with fused bias / per-step row bias (time embedding) / residual / ReLU / ReLU-backward mask.
// Split-K writes fp32 partial slabs that a second kernel reduces through the same epilogue.
#include "common.h"

struct ConvGemmParams {
  const bf16* x;
  const bf16* x2;       // channels >= c1 come from x2 (two-source concat, UNet skip connections)
  int ldx, ldx2, c1;
  int nb, hin, win, cin;
  int hout, wout;
  int kh, kw, stride, pad;
  int mode;             // 0: direct conv; 1: nearest-upsample (hin->hout) then conv s1; 2: transposed s2 gather
  const bf16* w;        // [cout][ktot]
  int ktot, cout;
  const float* bias;    // [cout]
  const bf16* rowbias;  // [*][rowbias_ld], row selected by *rowbias_idx (per-step time embedding)
  const int* rowbias_idx;
  int rowbias_ld;
  const bf16* resid;
  int ldr;
  const bf16* mask;     // ReLU backward: out *= (mask > 0)
  int ldmask;
  int act;              // 0 none, 1 relu
  bf16* y;
  int ldy;
  float* ws;            // split-K partial slabs [splits][M][npad]
  long ws_bytes;
  int splits, kps, npad;
};

namespace {

__device__ __forceinline__ void epilogue_store(const ConvGemmParams& p, long m, int c, float* v) {
  const bool full = (c + 8 <= p.cout);
  const int cnt = full ? 8 : (p.cout - c);
  if (p.bias) {
#pragma unroll
    for (int i = 0; i < 8; ++i) if (i < cnt) v[i] += p.bias[c + i];
  }
  if (p.rowbias) {
    const bf16* rb = p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) if (i < cnt) v[i] = (float)(bf16)v[i] + (float)rb[i];
  }
  if (p.resid) {
    const bf16* r = p.resid + m * p.ldr + c;
    if (full) {
      float rf[8];
      load8(r, rf);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + rf[i];
    } else {
      for (int i = 0; i < cnt; ++i) v[i] = (float)(bf16)v[i] + (float)r[i];
    }
  }
  if (p.act == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
  }
  if (p.mask) {
    const bf16* mk = p.mask + m * p.ldmask + c;
    if (full) {
      float mf[8];
      load8(mk, mf);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = mf[i] > 0.0f ? v[i] : 0.0f;
    } else {
      for (int i = 0; i < cnt; ++i) v[i] = (float)mk[i] > 0.0f ? v[i] : 0.0f;
    }
  }
  bf16* out = p.y + m * p.ldy + c;
  if (full) {
    store8(out, v);
  } else {
    for (int i = 0; i < cnt; ++i) out[i] = (bf16)v[i];
  }
}

template <int BM, int BN>
struct Smem {
  static constexpr int STAGE = (BM + BN) * 64 * 2;
  static constexpr int EPI = BM * (BN + 4) * 4;
  static constexpr int BYTES = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
};

template <int BM, int BN, bool SMALLC>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const ConvGemmParams p) {
  constexpr int AP = BM / 32;  // A pieces (16 B) per thread per k-chunk
  constexpr int BP = BN / 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const long hwo = (long)p.hout * p.wout;
  const long M = (long)p.nb * hwo;
  const int tiles_n = (p.cout + BN - 1) / BN;

  // bijective XCD-aware remap: blocks sharing an XCD (b % 8) get a contiguous tile range
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int lb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = lb / tiles_n, tn = lb - tm * tiles_n;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;

  const int nk = p.ktot >> 6;
  const int kc_begin = blockIdx.y * p.kps;
  const int kc_end = min(nk, kc_begin + p.kps);

  // per-thread A-row metadata
  const int piece = tid & 7;
  int a_n[AP], a_y[AP], a_x[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const long m = m0 + (tid >> 3) + 32 * i;
    if (m < M) {
      const int n = (int)(m / hwo);
      const int rem = (int)(m - (long)n * hwo);
      const int oy = rem / p.wout, ox = rem - (rem / p.wout) * p.wout;
      a_n[i] = n;
      if (p.mode == 0) {
        a_y[i] = oy * p.stride - p.pad;
        a_x[i] = ox * p.stride - p.pad;
      } else {
        a_y[i] = oy - p.pad;
        a_x[i] = ox - p.pad;
      }
    } else {
      a_n[i] = 0;
      a_y[i] = -(1 << 28);
      a_x[i] = -(1 << 28);
    }
  }
  const int cch = SMALLC ? 1 : (p.cin >> 6);

  uint4 ra[AP], rb[BP];

  auto load_chunk = [&](int kc) {
    int ky = 0, kx = 0, c = 0;
    bool tap_ok = true;
    if (!SMALLC) {
      const int tap = kc / cch;
      c = (kc - tap * cch) * 64 + piece * 8;
      ky = tap / p.kw;
      kx = tap - ky * p.kw;
    } else {
      const int k = kc * 64 + piece * 8;
      const int tap = k / p.cin;
      c = k - tap * p.cin;
      tap_ok = tap < p.kh * p.kw;
      ky = tap / p.kw;
      kx = tap - ky * p.kw;
    }
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      int iy = a_y[i] + ky, ix = a_x[i] + kx;
      bool ok = tap_ok;
      if (p.mode == 0) {
        ok = ok && iy >= 0 && iy < p.hin && ix >= 0 && ix < p.win;
      } else if (p.mode == 1) {
        ok = ok && iy >= 0 && iy < p.hout && ix >= 0 && ix < p.wout;
        iy = (int)(((long)iy * p.hin) / p.hout);
        ix = (int)(((long)ix * p.win) / p.wout);
      } else {
        ok = ok && iy >= 0 && ix >= 0 && !(iy & 1) && !(ix & 1);
        iy >>= 1;
        ix >>= 1;
        ok = ok && iy < p.hin && ix < p.win;
      }
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ok) {
        const long pix = ((long)a_n[i] * p.hin + iy) * p.win + ix;
        const bf16* src = (c < p.c1) ? (p.x + pix * p.ldx + c) : (p.x2 + pix * p.ldx2 + (c - p.c1));
        v = *reinterpret_cast<const uint4*>(src);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int j = 0; j < BP; ++j) {
      const int co = n0 + (tid >> 3) + 32 * j;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (co < p.cout) v = *reinterpret_cast<const uint4*>(p.w + (long)co * p.ktot + kc * 64 + piece * 8);
      rb[j] = v;
    }
  };

  auto store_chunk = [&](int stage) {
    char* sa = smem + stage * Smem<BM, BN>::STAGE;
    char* sb = sa + BM * 128;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<uint4*>(sa + row * 128 + ((piece ^ (row & 7)) << 4)) = ra[i];
    }
#pragma unroll
    for (int j = 0; j < BP; ++j) {
      const int row = (tid >> 3) + 32 * j;
      *reinterpret_cast<uint4*>(sb + row * 128 + ((piece ^ (row & 7)) << 4)) = rb[j];
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kc_begin < kc_end) {
    load_chunk(kc_begin);
    store_chunk(0);
  }
  __syncthreads();
  for (int kc = kc_begin; kc < kc_end; ++kc) {
    const int cur = (kc - kc_begin) & 1;
    const bool more = kc + 1 < kc_end;
    if (more) load_chunk(kc + 1);
    const char* sa = smem + cur * Smem<BM, BN>::STAGE;
    const char* sb = sa + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(sa + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_chunk(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS fp32 tile -> 8-wide coalesced rows
  float* cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * WM + i * 16 + (lane >> 4) * 4 + e;
        const int col = wn * WN + j * 16 + (lane & 15);
        cs[row * LDC + col] = acc[i][j][e];
      }
  __syncthreads();
  constexpr int GPR = BN / 8;
  for (int g = tid; g < BM * GPR; g += 256) {
    const int row = g / GPR, cg = g - (g / GPR) * GPR;
    const long m = m0 + row;
    const int c = n0 + cg * 8;
    if (m >= M || c >= p.cout) continue;
    float v[8];
    const float4 lo = *reinterpret_cast<const float4*>(cs + row * LDC + cg * 8);
    const float4 hi = *reinterpret_cast<const float4*>(cs + row * LDC + cg * 8 + 4);
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    if (p.splits > 1) {
      float* dst = p.ws + ((long)blockIdx.y * M + m) * p.npad + c;
      *reinterpret_cast<float4*>(dst) = lo;
      *reinterpret_cast<float4*>(dst + 4) = hi;
    } else {
      epilogue_store(p, m, c, v);
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const ConvGemmParams p, long M) {
  const int gpr = p.npad / 8;
  const long total = M * gpr;
  for (long g = blockIdx.x * 256L + threadIdx.x; g < total; g += (long)gridDim.x * 256) {
    const long m = g / gpr;
    const int c = (int)(g - m * gpr) * 8;
    if (c >= p.cout) continue;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < p.splits; ++s) {
      const float* src = p.ws + ((long)s * M + m) * p.npad + c;
      const float4 lo = *reinterpret_cast<const float4*>(src);
      const float4 hi = *reinterpret_cast<const float4*>(src + 4);
      v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w;
      v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
    }
    epilogue_store(p, m, c, v);
  }
}

template <int BM, int BN, bool SMALLC>
int launch_tile(ConvGemmParams& p, long M, hipStream_t stream) {
  const int tiles = (int)((M + BM - 1) / BM) * ((p.cout + BN - 1) / BN);
  const int nk = p.ktot / 64;
  p.npad = ((p.cout + BN - 1) / BN) * BN;
  int splits = 1;
  if (p.ws != nullptr && tiles < 200 && nk >= 8) {
    splits = (400 + tiles - 1) / tiles;
    splits = min(splits, nk / 4);
    splits = min(splits, 16);
    while (splits > 1 && (long)splits * M * p.npad * 4 > p.ws_bytes) --splits;
    splits = max(splits, 1);
  }
  p.kps = (nk + splits - 1) / splits;
  splits = (nk + p.kps - 1) / p.kps;
  p.splits = splits;
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, SMALLC>), dim3(tiles, splits), dim3(256), 0, stream, p);
  if (splits > 1) {
    const long groups = M * (p.npad / 8);
    const long nbl = (groups + 255) / 256;
    const int blocks = (int)(nbl < 8192 ? nbl : 8192);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, stream, p, M);
  }
  DC_CHECK_LAUNCH();
  return DC_OK;
}

}  // namespace

#include "../../include/dcamd.h"

extern "C" int dc_conv_gemm(const dc_conv_desc* d, void* stream) {
  if (!d || !d->x || !d->w || !d->y) return DC_ERR_ARG;
  ConvGemmParams p;
  p.x = (const bf16*)d->x;
  p.x2 = (const bf16*)(d->x2 ? d->x2 : d->x);
  p.ldx = d->ldx;
  p.ldx2 = d->x2 ? d->ldx2 : d->ldx;
  p.c1 = d->x2 ? d->c1 : (1 << 30);
  p.nb = d->nb; p.hin = d->hin; p.win = d->win; p.cin = d->cin;
  p.hout = d->hout; p.wout = d->wout;
  p.kh = d->kh; p.kw = d->kw; p.stride = d->stride; p.pad = d->pad; p.mode = d->mode;
  p.w = (const bf16*)d->w; p.ktot = d->ktot; p.cout = d->cout;
  p.bias = d->bias;
  p.rowbias = (const bf16*)d->rowbias; p.rowbias_idx = d->rowbias_idx; p.rowbias_ld = d->rowbias_ld;
  p.resid = (const bf16*)d->resid; p.ldr = d->ldr;
  p.mask = (const bf16*)d->mask; p.ldmask = d->ldmask;
  p.act = d->act;
  p.y = (bf16*)d->y; p.ldy = d->ldy;
  p.ws = d->ws; p.ws_bytes = d->ws_bytes;
  p.splits = 1; p.kps = 0; p.npad = 0;
  // shape / alignment contract (host pads channels, see DESIGN.md "layouts")
  if (p.ktot % 64 != 0 || p.ktot < p.kh * p.kw * p.cin) return DC_ERR_ARG;
  if (p.cin % 8 != 0 || p.cout <= 0 || p.nb <= 0 || p.hout <= 0 || p.wout <= 0) return DC_ERR_ARG;
  if (p.rowbias && !p.rowbias_idx) return DC_ERR_ARG;
  if (p.mode < 0 || p.mode > 2) return DC_ERR_ARG;
  if (p.mode == 2 && p.kh != 3) return DC_ERR_ARG;
  const bool smallc = (p.cin % 64) != 0;
  if (d->x2 && (smallc || p.c1 % 64 != 0)) return DC_ERR_ARG;
  if ((p.ldx | p.ldx2 | p.ldy) % 8 != 0) return DC_ERR_ALIGN;
  if (p.resid && p.ldr % 8 != 0) return DC_ERR_ALIGN;
  if (p.mask && p.ldmask % 8 != 0) return DC_ERR_ALIGN;
  if (((uintptr_t)p.x | (uintptr_t)p.x2 | (uintptr_t)p.w | (uintptr_t)p.y) & 15) return DC_ERR_ALIGN;
  if (((uintptr_t)p.resid | (uintptr_t)p.mask) & 15) return DC_ERR_ALIGN;
  const long M = (long)p.nb * p.hout * p.wout;
  hipStream_t s = (hipStream_t)stream;
  const bool narrow = (p.cout <= 64) || (((p.cout + 63) / 64) * 64 < ((p.cout + 127) / 128) * 128);
  if (smallc) {
    return narrow ? launch_tile<128, 64, true>(p, M, s) : launch_tile<128, 128, true>(p, M, s);
  }
  return narrow ? launch_tile<128, 64, false>(p, M, s) : launch_tile<128, 128, false>(p, M, s);
}
