// Host-side (CPU) helpers shared by both hosts of the sampler -- the Python pipeline (pipeline.py, unet.py,
// weights.py call them through ctypes) and the native session (session.cpp) -- so that the per-call tables
// and load-time constants they feed to the kernels are the same bits on either host.
//   dc_schedule_tables       DDIMScheduler (scaled_linear 0.00085..0.012, v_prediction, set_alpha_to_one=False,
//                            timestep_spacing="trailing"; marigold_dc.py:800, 814, 823-826, 902-904, predict.py:491-494)
//                            reduced to per-step scalars, and torch.optim.Adam's bias corrections (:783, 897)
//   dc_timestep_embedding    diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0), fp32
//   dc_fold_cross_attention  attn2 with the constant 2-token empty-prompt context folded to (U, D, c0)
//   dc_fold_layernorm        a LayerNorm folded into the linear that consumes it (include/dcamd.h dc_ln_fuse)
//   dc_fold_linear_pair      FF2 and proj_out of a transformer block folded into one two-source linear
//   dc_conv_pick             the tuned GEMM variant of a conv shape, nearest tuned shape for shapes not in the table
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/dcamd.h"

namespace {
inline float round_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return f;
  u += 0x7fffu + ((u >> 16) & 1u);
  u &= 0xffff0000u;
  float r;
  memcpy(&r, &u, 4);
  return r;
}
}  // namespace

extern "C" int dc_schedule_tables(int steps, double lr_latent, double lr_scaling, int opt, long long* timesteps,
                                  float* coef, float* adam) {
  constexpr int T = 1000;
  if (steps <= 0 || steps > T || opt < 0 || opt > 2 || !timesteps || !coef || !adam) return 1;
  // betas = linspace(sqrt(0.00085), sqrt(0.012), T, fp32) ** 2; alphas_cumprod = cumprod(1 - betas)
  // (torch's linspace: start + step * i below the midpoint, end - step * (T - 1 - i) above; cumprod
  // accumulates in double and stores fp32)
  const float start = (float)std::sqrt(0.00085), end = (float)std::sqrt(0.012);
  const float step = (end - start) / (float)(T - 1);
  std::vector<float> ac(T);
  double acc = 1.0;
  for (int i = 0; i < T; ++i) {
    volatile float prod = i < T / 2 ? step * (float)i : step * (float)(T - 1 - i);  // no fma contraction
    const float lin = i < T / 2 ? start + prod : end - prod;
    volatile float beta = lin * lin;
    acc *= (double)(1.0f - beta);
    ac[i] = (float)acc;
  }
  // trailing timesteps: round(arange(T, 0, -T / steps)) - 1 (numpy: start + i * delta, round half to even)
  const double ratio = (double)T / steps;
  const double delta = ((double)T + (-ratio)) - (double)T;
  for (int s = 0; s < steps; ++s) {
    const double v = (double)T + s * delta;
    const long long t = (long long)std::nearbyint(v) - 1;
    if (t < 0 || t >= T) return 1;
    timesteps[s] = t;
    const float a = ac[t];
    const long long prev = t - T / steps;
    const float ap = prev >= 0 ? ac[prev] : ac[0];
    const float b = 1.0f - a;
    coef[4 * s + 0] = std::sqrt(a);
    coef[4 * s + 1] = std::sqrt(b);
    coef[4 * s + 2] = std::sqrt(ap);
    coef[4 * s + 3] = std::sqrt(1.0f - ap);
    if (opt == 0) {
      // Adam: Python doubles lr / (1 - beta1^k), (1 - beta2^k) ** 0.5, cast to fp32 (foreach kernels)
      const int k = s + 1;
      const double bc1 = 1.0 - std::pow(0.9, k), bc2 = 1.0 - std::pow(0.999, k);
      adam[4 * s + 0] = (float)(lr_latent / bc1);
      adam[4 * s + 1] = (float)std::pow(bc2, 0.5);
      adam[4 * s + 2] = (float)(lr_scaling / bc1);
      adam[4 * s + 3] = 0.0f;
    } else {
      adam[4 * s + 0] = (float)lr_latent;
      adam[4 * s + 1] = 0.0f;
      adam[4 * s + 2] = (float)lr_scaling;
      adam[4 * s + 3] = 0.0f;
    }
  }
  return 0;
}

extern "C" int dc_timestep_embedding(const long long* timesteps, int n, int dim, float* out) {
  if (n <= 0 || dim <= 1 || (dim & 1) || !timesteps || !out) return 1;
  const int half = dim / 2;
  const float nlog = (float)(-std::log(10000.0));
  std::vector<float> freq(half);
  for (int i = 0; i < half; ++i) {
    volatile float e = nlog * (float)i;
    freq[i] = std::exp(e / (float)half);
  }
  for (int r = 0; r < n; ++r) {
    const float t = (float)timesteps[r];
    for (int i = 0; i < half; ++i) {
      const float e = t * freq[i];
      out[(long)r * dim + i] = std::cos(e);          // flip_sin_to_cos: [cos | sin]
      out[(long)r * dim + half + i] = std::sin(e);
    }
  }
  return 0;
}

extern "C" int dc_fold_layernorm(const float* w, int cout, int k, const float* gamma, const float* beta,
                                 const float* bias, void* wf, float* csum, float* cbias) {
  // W' = bf16(W[n][k] gamma[k]); csum[n] = sum_k W'[n][k] (of the rounded W', so that the kernel's
  // x . W' - mean csum equals (x - mean) . W' up to fp32 rounding); cbias[n] = sum_k W[n][k] beta[k] + bias[n]
  // (double, in k order: both hosts get the same bits)
  if (!w || !gamma || !beta || !wf || !csum || !cbias || cout <= 0 || k <= 0) return 1;
  uint16_t* o = static_cast<uint16_t*>(wf);
  for (int n = 0; n < cout; ++n) {
    double cs = 0.0, cb = 0.0;
    for (int i = 0; i < k; ++i) {
      const float wv = round_bf16(w[(size_t)n * k + i]);
      const float f = round_bf16(wv * round_bf16(gamma[i]));
      uint32_t u;
      memcpy(&u, &f, 4);
      o[(size_t)n * k + i] = (uint16_t)(u >> 16);
      cs += (double)f;
      cb += (double)wv * (double)round_bf16(beta[i]);
    }
    csum[n] = (float)cs;
    cbias[n] = (float)(cb + (bias ? (double)round_bf16(bias[n]) : 0.0));
  }
  return 0;
}

extern "C" int dc_fold_linear_pair(const float* w2, const float* b2, int c, int k2, const float* wp, const float* bp,
                                   void* wf, void* wd, float* bias) {
  if (!w2 || !b2 || !wp || !bp || !wf || !wd || !bias || c <= 0 || k2 <= 0) return 1;
  const int kt = k2 + c;
  uint16_t* of = static_cast<uint16_t*>(wf);
  uint16_t* od = static_cast<uint16_t*>(wd);
  auto bits = [](float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)(u >> 16);
  };
  std::vector<double> w2d;
  try {
    w2d.resize((size_t)c * k2);
  } catch (...) {
    return 1;
  }
  for (size_t e = 0; e < w2d.size(); ++e) w2d[e] = (double)round_bf16(w2[e]);
  std::atomic<int> failed{0};
  auto rows = [&](int r0, int r1) {
    std::vector<double> acc;
    try {
      acc.resize((size_t)k2);
    } catch (...) {   // a thread body must not throw (std::terminate)
      failed = 1;
      return;
    }
    for (int i = r0; i < r1; ++i) {   // row i of Wp W2: sum_m Wp[i][m] W2[m][.], m ascending
      std::fill(acc.begin(), acc.end(), 0.0);
      for (int m = 0; m < c; ++m) {
        const double a = (double)round_bf16(wp[(size_t)i * c + m]);
        const double* w2m = w2d.data() + (size_t)m * k2;
        for (int j = 0; j < k2; ++j) acc[j] += a * w2m[j];
      }
      for (int j = 0; j < k2; ++j) {
        const uint16_t b = bits(round_bf16((float)acc[j]));
        of[(size_t)i * kt + j] = b;
        od[(size_t)j * c + i] = b;
      }
      for (int j = 0; j < c; ++j) {
        const uint16_t b = bits(round_bf16(wp[(size_t)i * c + j]));
        of[(size_t)i * kt + k2 + j] = b;
        od[(size_t)(k2 + j) * c + i] = b;
      }
      double bb = (double)round_bf16(bp[i]);
      for (int m = 0; m < c; ++m) bb += (double)round_bf16(wp[(size_t)i * c + m]) * (double)round_bf16(b2[m]);
      bias[i] = (float)bb;
    }
  };
  // nothing may cross the C ABI: a failed thread creation runs the remaining rows on this thread (each row is summed
  // in a fixed order, so the bits do not depend on the split), and an allocation failure returns nonzero
  try {
    const int nt = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    int done = 0;   // rows [0, done) handed to threads
    for (int t = 0; t < nt; ++t) {
      const int r0 = (int)((long)c * t / nt), r1 = (int)((long)c * (t + 1) / nt);
      if (r1 <= r0) continue;
      try {
        th.emplace_back(rows, r0, r1);
        done = r1;
      } catch (const std::system_error&) {
        break;
      }
    }
    for (auto& x : th) x.join();
    if (done < c) rows(done, c);
  } catch (...) {
    return 1;
  }
  return failed ? 1 : 0;
}

extern "C" int dc_fold_cross_attention(const float* wq, const float* wk, const float* wv, const float* wo,
                                       const float* bo, const float* ctx, int ntok, int inner, int c, int cross,
                                       int cout, int heads, float* U, float* D, float* c0) {
  // softmax over the 2 context tokens: p0 = sigmoid(q . (k0 - k1) / sqrt(hd)); out = v1 + p0 (v0 - v1) per head:
  //   U_h = Wq_h^T (k0_h - k1_h) / sqrt(hd),  D_h = Wo_h (v0_h - v1_h),  c0 = Wo v1 + bo
  // in double from bf16-rounded weights; k, v rounded to bf16 as the reference's to_k / to_v produce them
  if (ntok != 2 || heads <= 0 || inner <= 0 || inner % heads || c <= 0 || cross <= 0 || cout <= 0) return 1;
  if (!wq || !wk || !wv || !wo || !bo || !ctx || !U || !D || !c0) return 1;
  const int hd = inner / heads;
  std::vector<double> k(2 * (size_t)inner), v(2 * (size_t)inner);
  for (int t = 0; t < 2; ++t)
    for (int j = 0; j < inner; ++j) {
      double sk = 0.0, sv = 0.0;
      for (int i = 0; i < cross; ++i) {
        const double ci = round_bf16(ctx[(size_t)t * cross + i]);
        sk += ci * round_bf16(wk[(size_t)j * cross + i]);
        sv += ci * round_bf16(wv[(size_t)j * cross + i]);
      }
      k[(size_t)t * inner + j] = round_bf16((float)sk);
      v[(size_t)t * inner + j] = round_bf16((float)sv);
    }
  const double scale = 1.0 / std::sqrt((double)hd);
  for (int h = 0; h < heads; ++h) {
    for (int col = 0; col < c; ++col) {
      double s = 0.0;
      for (int j = h * hd; j < (h + 1) * hd; ++j)
        s += (double)round_bf16(wq[(size_t)j * c + col]) * (k[j] - k[(size_t)inner + j]);
      U[(size_t)h * c + col] = (float)(s * scale);
    }
    for (int o = 0; o < cout; ++o) {
      double s = 0.0;
      for (int j = h * hd; j < (h + 1) * hd; ++j)
        s += (double)round_bf16(wo[(size_t)o * inner + j]) * (v[j] - v[(size_t)inner + j]);
      D[(size_t)h * cout + o] = (float)s;
    }
  }
  for (int o = 0; o < cout; ++o) {
    double s = 0.0;
    for (int j = 0; j < inner; ++j) s += (double)round_bf16(wo[(size_t)o * inner + j]) * v[(size_t)inner + j];
    c0[o] = (float)(s + (double)round_bf16(bo[o]));
  }
  return 0;
}

extern "C" int dc_conv_pick(const int* keys, const int* choices, int n, const int* key, int* out) {
  if (!out) return 1;
  out[0] = 0;
  out[1] = 0;
  if (!keys || !choices || !key || n <= 0) return 1;
  auto lg = [](long long v) { return std::log2((double)(v > 0 ? v : 1)); };
  const long long m = (long long)key[1] * key[5] * key[6];
  const double lm = lg(m), ln = lg(key[7]), lk = lg(key[11]);
  int best = -1;
  double best_d = 0.0;
  for (int i = 0; i < n; ++i) {
    const int* k = keys + 12 * (long)i;
    if (std::memcmp(k, key, 12 * sizeof(int)) == 0) {
      best = i;
      break;
    }
    if (k[0] != key[0] || k[8] != key[8] || k[9] != key[9] || k[10] != key[10]) continue;
    const double d = 4.0 * std::fabs(lg((long long)k[1] * k[5] * k[6]) - lm) + std::fabs(lg(k[7]) - ln) +
                     std::fabs(lg(k[11]) - lk);
    if (best < 0 || d < best_d) {
      best = i;
      best_d = d;
    }
  }
  if (best < 0) return 1;
  out[0] = choices[2 * best];
  out[1] = choices[2 * best + 1];
  return 0;
}
