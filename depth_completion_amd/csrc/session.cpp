// Native session: the whole guided sampler behind the C ABI (include/dcamd.h, "session" section), for hosts
// that are not Python.  SURVEY.md §8(b): dc_create / dc_destroy / dc_load_weights / dc_encode /
// dc_guided_sample / dc_decode_dense (+ dc_complete = marigold_dc.py:467-985 in one call).
//
// It is the C++ twin of the Python host (depth_completion_amd/pipeline.py, unet.py, taesd.py, weights.py):
// the same weight packing, the same buffers and the same launch sequence of the same kernels with the same
// arguments and the same GEMM variant table, so its results equal the Python pipeline's bitwise
// (tests/test_gpu_session.py).  Scope: the predict.py default path -- guided per-step optimisation of the
// latents and the learned affine with the l1 + l2 point losses, TAESD, norm const / minmax, any projection /
// inv / interpolation / optimiser -- one guided step captured as a hipGraph and replayed for every timestep.
// The other modes (closed form, per-input, KL, edge / smooth, AutoencoderKL, percentile) stay on the Python
// host over the same kernels.
//
// Weights come from a local directory in the diffusers layout (no network): unet/config.json +
// unet/diffusion_pytorch_model.safetensors, taesd/diffusion_pytorch_model.safetensors, and
// empty_text_embedding.safetensors ("embedding" [1, 2, cross_attention_dim], the CLIP encoding of the empty
// prompt, marigold_dc.py:663-674, written once by the Python host's from_pretrained).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/dcamd.h"
#include "json_mini.h"
#include "safetensors_mini.h"

namespace {

constexpr int kOK = 0, kErrArg = 1, kErrLaunch = 2;

struct DcError : std::runtime_error {
  int code;
  DcError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define DCK(expr)                                                                            \
  do {                                                                                       \
    const int _st = (expr);                                                                  \
    if (_st != 0) throw DcError(_st, std::string(#expr).substr(0, std::string(#expr).find('(')) + " failed"); \
  } while (0)
#define HIPK(expr)                                                                              \
  do {                                                                                          \
    const hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) throw DcError(kErrLaunch, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------ bf16 on the host (torch's rounding)
inline uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float round_bf16(float f) { return dcst::bf2f(f2bf(f)); }
// ------------------------------------------------------------------ safetensors (read-only mmap, validated)
using dcst::bf2f;
using dcst::HostTensor;
using dcst::SafeTensors;

std::string read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return std::string();
  std::string s;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  fclose(f);
  return s;
}

// ------------------------------------------------------------------ device memory owned by the session
// Move-only: `x = DevMem()` frees x's blocks (a copy would drop them without freeing).
struct DevMem {
  std::vector<void*> blocks;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  DevMem(DevMem&& o) noexcept : blocks(std::move(o.blocks)) { o.blocks.clear(); }
  DevMem& operator=(DevMem&& o) noexcept {
    if (this != &o) {
      release();
      blocks = std::move(o.blocks);
      o.blocks.clear();
    }
    return *this;
  }
  ~DevMem() { release(); }
  void release() {
    for (void* p : blocks) (void)hipFree(p);
    blocks.clear();
  }
  void* alloc(size_t bytes, bool zero = true) {
    void* p = nullptr;
    HIPK(hipMalloc(&p, bytes < 16 ? 16 : bytes));
    if (zero) HIPK(hipMemset(p, 0, bytes < 16 ? 16 : bytes));
    blocks.push_back(p);
    return p;
  }
  template <typename T>
  T* upload(const std::vector<T>& v) {
    T* p = (T*)alloc(v.size() * sizeof(T), false);
    HIPK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
  }
};

// row buffer view: bf16 [rows][ld] (a column offset is folded into p)
struct RB {
  void* p = nullptr;
  int ld = 0;
  RB() = default;
  RB(void* p_, int ld_) : p(p_), ld(ld_) {}
  RB col(int c) const { return RB((char*)p + (size_t)c * 2, ld); }
};

// ------------------------------------------------------------------ weights (weights.py)
std::vector<uint16_t> to_bf16(const std::vector<float>& v) {
  std::vector<uint16_t> o(v.size());
  for (size_t i = 0; i < v.size(); ++i) o[i] = f2bf(v[i]);
  return o;
}

// [co][ci][kh][kw] -> [co][ktot] with K = (ky, kx, cin padded to cp), ktot padded to 64 (pack_conv)
std::vector<float> pack_conv(const std::vector<float>& w, int co, int ci, int kh, int kw, int cp, int* ktot) {
  const int k = kh * kw * cp;
  const int kt = (k + 63) / 64 * 64;
  std::vector<float> t((size_t)co * kt, 0.0f);
  for (int o = 0; o < co; ++o)
    for (int y = 0; y < kh; ++y)
      for (int x = 0; x < kw; ++x)
        for (int i = 0; i < ci; ++i) t[(size_t)o * kt + (y * kw + x) * cp + i] = w[(((size_t)o * ci + i) * kh + y) * kw + x];
  *ktot = kt;
  return t;
}

struct ConvW {
  int cout = 0, cin = 0, kh = 0, kw = 0, stride = 1, ktot_f = 0, ktot_d = 0;
  void* wf = nullptr;
  void* wd = nullptr;
  float* bias = nullptr;
};

struct LinearW {
  int cout = 0, cin = 0;
  void* wf = nullptr;  // [cout][cin]
  void* wd = nullptr;  // [cin][cout]
  float* bias = nullptr;
  // a LayerNorm folded in (weights.LnLinear, dc_ln_fuse): wf / wd are the gamma-scaled weights, bias is NULL
  float* csum = nullptr;
  float* cbias = nullptr;
  float eps = 0.0f;
};

struct NormW {
  float* gamma = nullptr;
  float* beta = nullptr;
  float eps = 1e-5f;
};

class Loader {
 public:
  Loader(const SafeTensors& st, DevMem& mem) : st_(st), mem_(mem) {}

  float* bias(const std::string& k) {
    HostTensor b = st_.get(k);
    for (float& v : b.data) v = round_bf16(v);
    return mem_.upload(b.data);
  }
  // weights.Conv
  ConvW conv(const std::string& pre, bool has_bias, int stride = 1, int cin_pad = 0, bool dgrad = true,
             const std::vector<int>* dgrad_rows = nullptr, int dgrad_cout_pad = 0) {
    HostTensor w = st_.get(pre + ".weight");
    for (float& v : w.data) v = round_bf16(v);
    ConvW c;
    c.cout = (int)w.shape[0];
    c.cin = (int)w.shape[1];
    c.kh = (int)w.shape[2];
    c.kw = (int)w.shape[3];
    c.stride = stride;
    const int cp = cin_pad ? cin_pad : c.cin;
    c.wf = mem_.upload(to_bf16(pack_conv(w.data, c.cout, c.cin, c.kh, c.kw, cp, &c.ktot_f)));
    if (has_bias) c.bias = bias(pre + ".bias");
    if (dgrad) {
      // W'[cin][cout][ky][kx] = W[cout][cin][kh-1-ky][kw-1-kx], rows selected, cout padded (pack_conv_dgrad)
      std::vector<int> rows;
      if (dgrad_rows) rows = *dgrad_rows;
      else for (int i = 0; i < c.cin; ++i) rows.push_back(i);
      const int nr = (int)rows.size();
      std::vector<float> wd((size_t)nr * c.cout * c.kh * c.kw);
      for (int r = 0; r < nr; ++r)
        for (int o = 0; o < c.cout; ++o)
          for (int y = 0; y < c.kh; ++y)
            for (int x = 0; x < c.kw; ++x)
              wd[(((size_t)r * c.cout + o) * c.kh + y) * c.kw + x] =
                  w.data[(((size_t)o * c.cin + rows[r]) * c.kh + (c.kh - 1 - y)) * c.kw + (c.kw - 1 - x)];
      const int cpd = dgrad_cout_pad ? dgrad_cout_pad : c.cout;
      c.wd = mem_.upload(to_bf16(pack_conv(wd, nr, c.cout, c.kh, c.kw, cpd, &c.ktot_d)));
    }
    return c;
  }
  // weights.Linear (rows optionally permuted: the GEGLU interleave)
  LinearW linear_from(HostTensor w, const float* b, bool dgrad = true) {
    for (float& v : w.data) v = round_bf16(v);
    LinearW l;
    l.cout = (int)w.shape[0];
    l.cin = (int)w.shape[1];
    l.wf = mem_.upload(to_bf16(w.data));
    if (b) {
      std::vector<float> bb(b, b + l.cout);
      for (float& v : bb) v = round_bf16(v);
      l.bias = mem_.upload(bb);
    }
    if (dgrad) {
      std::vector<float> t((size_t)l.cin * l.cout);
      for (int o = 0; o < l.cout; ++o)
        for (int i = 0; i < l.cin; ++i) t[(size_t)i * l.cout + o] = w.data[(size_t)o * l.cin + i];
      l.wd = mem_.upload(to_bf16(t));
    }
    return l;
  }
  // weights.LnLinear: the LayerNorm `norm_pre` folded into the linear (the shared host routine dc_fold_layernorm)
  LinearW linear_ln_from(HostTensor w, const float* b, const std::string& norm_pre, float eps) {
    HostTensor g = st_.get(norm_pre + ".weight"), be = st_.get(norm_pre + ".bias");
    LinearW l;
    l.cout = (int)w.shape[0];
    l.cin = (int)w.shape[1];
    l.eps = eps;
    std::vector<uint16_t> wf((size_t)l.cout * l.cin);
    std::vector<float> cs(l.cout), cb(l.cout);
    DCK(dc_fold_layernorm(w.data.data(), l.cout, l.cin, g.data.data(), be.data.data(), b, wf.data(), cs.data(),
                          cb.data()));
    l.wf = mem_.upload(wf);
    std::vector<uint16_t> t((size_t)l.cin * l.cout);
    for (int o = 0; o < l.cout; ++o)
      for (int i = 0; i < l.cin; ++i) t[(size_t)i * l.cout + o] = wf[(size_t)o * l.cin + i];
    l.wd = mem_.upload(t);
    l.csum = mem_.upload(cs);
    l.cbias = mem_.upload(cb);
    return l;
  }
  // weights.FoldedPair: FF2 and proj_out as one two-source linear over [gg | r2] (the shared host routine
  // dc_fold_linear_pair); wf [c][k2 + c], wd [k2 + c][c], bias fp32
  LinearW linear_pair(const std::string& ff2, const std::string& proj_out) {
    HostTensor w2 = st_.get(ff2 + ".weight"), b2 = st_.get(ff2 + ".bias");
    HostTensor wp = st_.get(proj_out + ".weight"), bp = st_.get(proj_out + ".bias");
    LinearW l;
    const int c = (int)w2.shape[0], k2 = (int)w2.shape[1];
    l.cout = c;
    l.cin = k2 + c;
    std::vector<uint16_t> wf((size_t)c * (k2 + c)), wd((size_t)(k2 + c) * c);
    std::vector<float> bias(c);
    DCK(dc_fold_linear_pair(w2.data.data(), b2.data.data(), c, k2, wp.data.data(), bp.data.data(), wf.data(),
                            wd.data(), bias.data()));
    l.wf = mem_.upload(wf);
    l.wd = mem_.upload(wd);
    l.bias = mem_.upload(bias);
    return l;
  }
  LinearW linear(const std::string& pre, bool has_bias, bool dgrad = true) {
    HostTensor w = st_.get(pre + ".weight");
    HostTensor b;
    if (has_bias) b = st_.get(pre + ".bias");
    return linear_from(std::move(w), has_bias ? b.data.data() : nullptr, dgrad);
  }
  NormW norm(const std::string& pre, float eps) {
    NormW n;
    HostTensor g = st_.get(pre + ".weight"), b = st_.get(pre + ".bias");
    for (float& v : g.data) v = round_bf16(v);
    for (float& v : b.data) v = round_bf16(v);
    n.gamma = mem_.upload(g.data);
    n.beta = mem_.upload(b.data);
    n.eps = eps;
    return n;
  }
  const SafeTensors& st() const { return st_; }
  DevMem& mem() { return mem_; }

 private:
  const SafeTensors& st_;
  DevMem& mem_;
};

// ------------------------------------------------------------------ tuned GEMM table (ops.load_tuned)
using ConvKey = std::tuple<int, int, int, int, int, int, int, int, int, int, int, int>;

struct Exec {
  hipStream_t stream = nullptr;
  float* ws = nullptr;  // fp32 scratch (split-K slabs, counters in its last 64 KB), zeroed once
  long long ws_bytes = 0;
  int* step = nullptr;  // device step counter
  std::map<ConvKey, std::pair<int, int>> tuned;
  // the tuned table in file order (dc_conv_pick picks the nearest tuned shape for a shape not in it, as the
  // Python host's ops.Ctx does), and the picks made so far
  std::vector<int> table_keys, table_choices;
  std::map<ConvKey, std::pair<int, int>> picked;
  bool nn = true;

  // ops.conv_gemm
  struct Conv {
    RB x;
    RB x2;
    int c1 = 0;
    int nb = 1, hin = 1, win = 1, cin = 0, hout = 1, wout = 1, cout = 0;
    int kh = 3, kw = 3, stride = 1, pad = 1, mode = 0;
    const void* w = nullptr;
    int ktot = 0;
    const float* bias = nullptr;
    const void* rowbias = nullptr;
    int rowbias_ld = 0;
    RB resid, mask;
    int act = 0;
    RB y;
    int geglu = 0;
    RB y2, aux;
    const int* rows = nullptr;
    int nrows = 0;
    const dc_gn_fuse* gn = nullptr;   // fused GroupNorm statistics (unet.py _gnf / _gn_bwd_fuse)
    const dc_ln_fuse* ln = nullptr;   // LayerNorm folded in (unet.py ln_fuse)
    int geglu_n = 0;                  // GEGLU backward on the first geglu_n columns only (the folded FF2 / proj_out)
  };
  void conv(const Conv& a) {
    const dc_conv_desc d = desc(a);
    DCK(dc_conv_gemm(&d, stream));
  }
  // the descriptor of one call, its variant chosen as ops.conv_desc chooses it
  dc_conv_desc desc(const Conv& a) {
    dc_conv_desc d;
    memset(&d, 0, sizeof d);
    d.x = a.x.p;
    d.ldx = a.x.ld;
    d.x2 = a.x2.p;
    d.ldx2 = a.x2.p ? a.x2.ld : 0;
    d.c1 = a.c1;
    d.nb = a.nb; d.hin = a.hin; d.win = a.win; d.cin = a.cin; d.hout = a.hout; d.wout = a.wout;
    d.kh = a.kh; d.kw = a.kw; d.stride = a.stride; d.pad = a.pad; d.mode = a.mode;
    d.w = a.w;
    d.ktot = a.ktot;
    d.cout = a.cout;
    d.bias = a.bias;
    d.rowbias = a.rowbias;
    d.rowbias_idx = a.rowbias ? step : nullptr;
    d.rowbias_ld = a.rowbias_ld;
    d.resid = a.resid.p;
    d.ldr = a.resid.p ? a.resid.ld : 0;
    d.mask = a.mask.p;
    d.ldmask = a.mask.p ? a.mask.ld : 0;
    d.act = a.act;
    d.y = a.y.p;
    d.ldy = a.y.ld;
    d.geglu = a.geglu;
    d.y2 = a.y2.p;
    d.ldy2 = a.y2.p ? a.y2.ld : 0;
    d.aux = a.aux.p;
    d.ldaux = a.aux.p ? a.aux.ld : 0;
    d.ws = ws;
    d.ws_bytes = ws_bytes;
    d.gn = a.gn;
    d.ln = a.ln;
    d.geglu_n = a.geglu_n;
    if (a.rows) {
      d.rows = a.rows;
      d.nrows = a.nrows;
      d.algo = 0;
      d.splitk = 0;
    } else {
      const ConvKey key{d.mode, d.nb, d.hin, d.win, d.cin, d.hout, d.wout, d.cout, d.kh, d.stride, d.x2 ? 1 : 0, d.ktot};
      auto it = tuned.find(key);
      if (it == tuned.end()) {
        it = picked.find(key);
        if (it == picked.end()) {
          int out[2] = {0, 0};
          const int kk[12] = {d.mode, d.nb, d.hin, d.win, d.cin, d.hout, d.wout, d.cout, d.kh, d.stride, d.x2 ? 1 : 0,
                              d.ktot};
          if (nn && !table_choices.empty())
            (void)dc_conv_pick(table_keys.data(), table_choices.data(), (int)(table_choices.size() / 2), kk, out);
          it = picked.emplace(key, std::make_pair(out[0], out[1])).first;
        }
      }
      d.algo = it->second.first;
      d.splitk = it->second.second;
    }
    return d;
  }
  // ops.linear
  void linear(RB x, const void* w, int k, int rows, int cout, RB y, const float* bias = nullptr, RB resid = RB(),
              const void* rowbias = nullptr, int rowbias_ld = 0, int geglu = 0, RB y2 = RB(), RB aux = RB(),
              const dc_gn_fuse* gn = nullptr, const dc_ln_fuse* ln = nullptr) {
    conv(lin(x, w, k, rows, cout, y, bias, resid, rowbias, rowbias_ld, geglu, y2, aux, gn, ln));
  }
  static Conv lin(RB x, const void* w, int k, int rows, int cout, RB y, const float* bias = nullptr, RB resid = RB(),
                  const void* rowbias = nullptr, int rowbias_ld = 0, int geglu = 0, RB y2 = RB(), RB aux = RB(),
                  const dc_gn_fuse* gn = nullptr, const dc_ln_fuse* ln = nullptr) {
    Conv a;
    a.x = x;
    a.nb = 1; a.hin = 1; a.win = rows; a.cin = k; a.hout = 1; a.wout = rows; a.cout = cout;
    a.kh = 1; a.kw = 1; a.stride = 1; a.pad = 0;
    a.w = w;
    a.ktot = k;
    a.bias = bias;
    a.resid = resid;
    a.rowbias = rowbias;
    a.rowbias_ld = rowbias_ld;
    a.y = y;
    a.geglu = geglu;
    a.y2 = y2;
    a.aux = aux;
    a.gn = gn;
    a.ln = ln;
    return a;
  }
  void groupnorm(RB x, int nb, int hw, int c, const NormW& n, bool silu, RB y, float* stats, RB x2 = RB(),
                 int c1 = 0) {
    DCK(dc_groupnorm_fwd(x.p, x.ld, x2.p, x2.p ? x2.ld : 0, c1, nb, hw, c, 32, n.eps, n.gamma, n.beta, silu ? 1 : 0,
                         y.p, y.ld, stats, ws, stream));
  }
  void groupnorm_bwd(RB x, int nb, int hw, int c, const NormW& n, bool silu, const float* stats, RB dy, RB dx,
                     RB x2 = RB(), int c1 = 0, RB add1 = RB(), RB add2 = RB()) {
    DCK(dc_groupnorm_bwd(x.p, x.ld, x2.p, x2.p ? x2.ld : 0, c1, nb, hw, c, 32, n.gamma, n.beta, silu ? 1 : 0, stats,
                         dy.p, dy.ld, dx.p, dx.ld, add1.p, add1.p ? add1.ld : 0, add2.p, add2.p ? add2.ld : 0, ws,
                         stream));
  }
  // ops.groupnorm_acc / ops.groupnorm_bwd_acc (fused statistics)
  void groupnorm_acc(RB x, int nb, int hw, int c, const NormW& n, bool silu, const long long* acc, RB y, float* stats,
                     RB x2 = RB(), int c1 = 0) {
    DCK(dc_groupnorm_fwd_acc(x.p, x.ld, x2.p, x2.p ? x2.ld : 0, c1, nb, hw, c, 32, n.eps, n.gamma, n.beta,
                             silu ? 1 : 0, acc, y.p, y.ld, stats, stream));
  }
  void groupnorm_bwd_acc(RB x, int nb, int hw, int c, const NormW& n, const float* stats, const long long* acc, RB dy,
                         RB dx, RB x2 = RB(), int c1 = 0, RB add1 = RB(), RB add2 = RB()) {
    DCK(dc_groupnorm_bwd_acc(x.p, x.ld, x2.p, x2.p ? x2.ld : 0, c1, nb, hw, c, 32, n.gamma, stats, acc, dy.p, dy.ld,
                             dx.p, dx.ld, add1.p, add1.p ? add1.ld : 0, add2.p, add2.p ? add2.ld : 0, stream));
  }
  void memset0(void* p, size_t bytes) { DCK(dc_memset_async(p, 0, (long long)bytes, stream)); }
};

void load_tuned(Exec& ex, const std::string& path) {
  const std::string s = read_file(path);
  if (s.empty()) return;
  dcjson::Value v = dcjson::parse(s);
  std::map<ConvKey, int> index;
  for (const auto& e : v.arr) {
    const auto& k = e.at("key").arr;
    if (k.size() != 12) continue;
    ConvKey key{(int)k[0].as_int(), (int)k[1].as_int(), (int)k[2].as_int(), (int)k[3].as_int(), (int)k[4].as_int(),
                (int)k[5].as_int(), (int)k[6].as_int(), (int)k[7].as_int(), (int)k[8].as_int(), (int)k[9].as_int(),
                (int)k[10].as_int(), (int)k[11].as_int()};
    const int algo = (int)e.at("algo").as_int(), splitk = (int)e.at("splitk").as_int();
    // a repeated key keeps its first position and takes the last value, as the Python host's dict does
    auto pos = index.find(key);
    if (pos != index.end()) {
      ex.table_choices[2 * pos->second] = algo;
      ex.table_choices[2 * pos->second + 1] = splitk;
    } else {
      index[key] = (int)(ex.table_choices.size() / 2);
      for (const auto& kv : k) ex.table_keys.push_back((int)kv.as_int());
      ex.table_choices.push_back(algo);
      ex.table_choices.push_back(splitk);
    }
    ex.tuned[key] = {algo, splitk};
  }
}

// ------------------------------------------------------------------ UNet (unet.py)
struct UNetCfg {
  std::vector<int> ch{320, 640, 1280, 1280};
  std::vector<int> heads{5, 10, 20, 20};
  std::vector<bool> down_attn{true, true, true, false};
  std::vector<bool> up_attn{false, true, true, true};
  int layers = 2;
  int cross = 1024;
};

struct ResnetW {
  NormW n1, n2;
  ConvW c1, c2, sc;
  bool has_sc = false;
  LinearW temb;
  int cin = 0, cout = 0;
  std::map<int, void*> temb_tables;  // per step count, kept for the session's lifetime (graph replay binds them)
  void* temb_table = nullptr;
};

struct TransformerW {
  int heads = 0, c = 0;
  NormW norm, ln1, ln2, ln3;
  LinearW proj_in, qkv, out, ff1;
  LinearW ffo;   // ff.net.2 + proj_out folded into one linear over [gg | r2] (dc_fold_linear_pair)
  float *U = nullptr, *D = nullptr, *c0 = nullptr;
  void* tabs = nullptr;  // MFMA operand tables of the folded cross-attention (dc_crossattn_prepare)
};

struct UNetW {
  UNetCfg cfg;
  ConvW conv_in, conv_out;
  LinearW t_lin1, t_lin2;
  struct Block {
    std::vector<ResnetW> res;
    std::vector<TransformerW> att;
    bool has_sampler = false;
    ConvW sampler;
  };
  std::vector<Block> down, up;
  std::vector<ResnetW> mid_res;
  TransformerW mid_attn;
  NormW norm_out;
  std::vector<ResnetW*> resnets() {
    std::vector<ResnetW*> r;
    for (auto& b : down) for (auto& x : b.res) r.push_back(&x);
    for (auto& x : mid_res) r.push_back(&x);
    for (auto& b : up) for (auto& x : b.res) r.push_back(&x);
    return r;
  }
};

ResnetW load_resnet(Loader& L, const std::string& pre) {
  ResnetW r;
  r.n1 = L.norm(pre + "norm1", 1e-5f);
  r.c1 = L.conv(pre + "conv1", true);
  r.temb = L.linear(pre + "time_emb_proj", true, false);
  r.n2 = L.norm(pre + "norm2", 1e-5f);
  r.c2 = L.conv(pre + "conv2", true);
  r.cin = r.c1.cin;
  r.cout = r.c1.cout;
  if (L.st().has(pre + "conv_shortcut.weight")) {
    r.has_sc = true;
    r.sc = L.conv(pre + "conv_shortcut", true);
  }
  return r;
}

TransformerW load_transformer(Loader& L, const std::string& pre, int heads, const std::vector<float>& ctx,
                              int ntok) {
  TransformerW t;
  t.heads = heads;
  t.norm = L.norm(pre + "norm", 1e-6f);
  t.proj_in = L.linear(pre + "proj_in", true);
  const std::string b = pre + "transformer_blocks.0.";
  t.ln1 = L.norm(b + "norm1", 1e-5f);
  t.ln2 = L.norm(b + "norm2", 1e-5f);
  t.ln3 = L.norm(b + "norm3", 1e-5f);
  const SafeTensors& st = L.st();
  HostTensor wq = st.get(b + "attn1.to_q.weight"), wk = st.get(b + "attn1.to_k.weight"),
             wv = st.get(b + "attn1.to_v.weight");
  HostTensor qkv;
  qkv.shape = {wq.shape[0] * 3, wq.shape[1]};
  qkv.data = wq.data;
  qkv.data.insert(qkv.data.end(), wk.data.begin(), wk.data.end());
  qkv.data.insert(qkv.data.end(), wv.data.begin(), wv.data.end());
  t.qkv = L.linear_from(std::move(qkv), nullptr);
  t.out = L.linear(b + "attn1.to_out.0", true);
  // folded cross-attention (weights.fold_cross_attention via the shared host routine)
  HostTensor q2 = st.get(b + "attn2.to_q.weight"), k2 = st.get(b + "attn2.to_k.weight"),
             v2 = st.get(b + "attn2.to_v.weight"), o2 = st.get(b + "attn2.to_out.0.weight"),
             bo2 = st.get(b + "attn2.to_out.0.bias");
  const int inner = (int)q2.shape[0], C = (int)q2.shape[1], cross = (int)k2.shape[1], cout = (int)o2.shape[0];
  std::vector<float> U((size_t)heads * C), D((size_t)heads * cout), c0(cout);
  DCK(dc_fold_cross_attention(q2.data.data(), k2.data.data(), v2.data.data(), o2.data.data(), bo2.data.data(),
                              ctx.data(), ntok, inner, C, cross, cout, heads, U.data(), D.data(), c0.data()));
  t.U = L.mem().upload(U);
  t.D = L.mem().upload(D);
  t.c0 = L.mem().upload(c0);
  t.tabs = L.mem().alloc((size_t)dc_crossattn_tables_bytes(heads, C), false);
  DCK(dc_crossattn_prepare(t.U, t.D, heads, C, t.tabs, nullptr));
  HIPK(hipDeviceSynchronize());
  // GEGLU projection with (h, gate) rows interleaved 8 + 8 (weights.geglu_interleave)
  HostTensor f1 = st.get(b + "ff.net.0.proj.weight"), f1b = st.get(b + "ff.net.0.proj.bias");
  const int nout = (int)f1.shape[0], kin = (int)f1.shape[1], inner_ff = nout / 2;
  HostTensor f1p;
  f1p.shape = f1.shape;
  f1p.data.resize(f1.data.size());
  std::vector<float> f1bp(nout);
  int r = 0;
  for (int blk = 0; blk < inner_ff; blk += 8) {
    for (int half = 0; half < 2; ++half)
      for (int j = 0; j < 8; ++j, ++r) {
        const int src = half * inner_ff + blk + j;
        memcpy(&f1p.data[(size_t)r * kin], &f1.data[(size_t)src * kin], (size_t)kin * 4);
        f1bp[r] = f1b.data[src];
      }
  }
  t.ff1 = L.linear_ln_from(std::move(f1p), f1bp.data(), b + "norm3", 1e-5f);   // norm3 folded
  t.ffo = L.linear_pair(b + "ff.net.2", pre + "proj_out");
  t.c = t.proj_in.cout;
  return t;
}

void load_unet(UNetW& u, Loader& L, const std::vector<float>& ctx, int ntok) {
  const UNetCfg& cfg = u.cfg;
  const std::vector<int> in_rows{4, 5, 6, 7};
  u.conv_in = L.conv("conv_in", true, 1, 0, true, &in_rows);
  u.t_lin1 = L.linear("time_embedding.linear_1", true, false);
  u.t_lin2 = L.linear("time_embedding.linear_2", true, false);
  const int nb = (int)cfg.ch.size();
  for (int i = 0; i < nb; ++i) {
    UNetW::Block b;
    for (int j = 0; j < cfg.layers; ++j) {
      b.res.push_back(load_resnet(L, "down_blocks." + std::to_string(i) + ".resnets." + std::to_string(j) + "."));
      if (cfg.down_attn[i])
        b.att.push_back(load_transformer(L, "down_blocks." + std::to_string(i) + ".attentions." + std::to_string(j) + ".",
                                         cfg.heads[i], ctx, ntok));
    }
    if (i < nb - 1) {
      b.has_sampler = true;
      b.sampler = L.conv("down_blocks." + std::to_string(i) + ".downsamplers.0.conv", true, 2);
    }
    u.down.push_back(std::move(b));
  }
  for (int j = 0; j < 2; ++j) u.mid_res.push_back(load_resnet(L, "mid_block.resnets." + std::to_string(j) + "."));
  u.mid_attn = load_transformer(L, "mid_block.attentions.0.", cfg.heads.back(), ctx, ntok);
  for (int i = 0; i < nb; ++i) {
    UNetW::Block b;
    const int rh = cfg.heads[nb - 1 - i];
    for (int j = 0; j < cfg.layers + 1; ++j) {
      b.res.push_back(load_resnet(L, "up_blocks." + std::to_string(i) + ".resnets." + std::to_string(j) + "."));
      if (cfg.up_attn[i])
        b.att.push_back(load_transformer(L, "up_blocks." + std::to_string(i) + ".attentions." + std::to_string(j) + ".",
                                         rh, ctx, ntok));
    }
    if (i < nb - 1) {
      b.has_sampler = true;
      b.sampler = L.conv("up_blocks." + std::to_string(i) + ".upsamplers.0.conv", true);
    }
    u.up.push_back(std::move(b));
  }
  u.norm_out = L.norm("conv_norm_out", 1e-5f);
  u.conv_out = L.conv("conv_out", true, 1, 0, true, nullptr, 8);
}

// UNetPlan: buffers + launch lists for one (frames, h, w)
class UNetPlan {
 public:
  UNetPlan(UNetW& net, Exec& ex, DevMem& mem, int nb, int h, int w) : net_(net), ex_(ex), mem_(mem), nb_(nb), h_(h), w_(w) {
    const int P = nb * h * w;
    x8 = buf(P, 8);
    v = buf(P, 8);
    dv = buf(P, 8);
    gx = buf(P, 8);
    // fused GroupNorm statistics (unet.py UNetPlan.fuse_gn): one accumulator per GroupNorm and direction in one
    // arena, zero-filled at the head of every forward
    const char* e = getenv("DC_GN_FUSE");
    fuse_gn_ = !(e && std::string(e) == "0");
    int n_res = 0, n_tr = 1;
    for (auto& b : net.down) { n_res += (int)b.res.size(); n_tr += (int)b.att.size(); }
    for (auto& b : net.up) { n_res += (int)b.res.size(); n_tr += (int)b.att.size(); }
    n_res += (int)net.mid_res.size();
    const int n_gn = 2 * (2 * n_res + n_tr + 1);
    gn_words_ = (size_t)dc_gn_acc_bytes(nb, 32) / 8;
    gn_arena_bytes_ = (size_t)n_gn * gn_words_ * 8;
    gn_arena_ = (long long*)mem_.alloc(gn_arena_bytes_);
    build_forward();
    build_backward();
  }
  void forward() { for (auto& f : fwd_) f(); }
  void backward() { for (auto& f : bwd_) f(); }
  RB x8, v, dv, gx;

 private:
  UNetW& net_;
  Exec& ex_;
  DevMem& mem_;
  int nb_, h_, w_;
  std::vector<std::function<void()>> fwd_, bwd_;
  struct TapeEntry {
    std::string kind;
    std::map<std::string, RB> b;
    std::map<std::string, float*> f;
    std::map<std::string, int> i;
    ResnetW* r = nullptr;
    TransformerW* t = nullptr;
    ConvW* cv = nullptr;
  };
  std::vector<TapeEntry> tape_;
  bool fuse_gn_ = true;
  long long* gn_arena_ = nullptr;
  size_t gn_words_ = 0, gn_arena_bytes_ = 0;
  int gn_next_ = 0;
  std::map<const void*, std::vector<dc_gn_target>> gn_targets_;       // output buffer -> GroupNorms it feeds
  std::map<const void*, std::unique_ptr<dc_gn_fuse>> gn_fuse_;        // built at the first call
  std::vector<std::unique_ptr<dc_gn_fuse>> gn_bwd_;                     // backward fuses (fixed at build)

  // unet.py _conv_fwd: a forward conv producing a.y, with the fused GroupNorm statistics of y's consumers
  void conv_fwd(Exec::Conv a) {
    a.gn = gnf(a.y);
    ex_.conv(a);
  }

  long long* gn_acc() {   // a GroupNorm site the arena was not sized for: fail, never hand out past its end
    if ((size_t)(gn_next_ + 1) * gn_words_ * 8 > gn_arena_bytes_)
      throw DcError(kErrArg, "GroupNorm accumulator arena exhausted (" + std::to_string(gn_next_) + " slots)");
    return gn_arena_ + (size_t)(gn_next_++) * gn_words_;
  }
  bool gn_pays(int hw, int c, bool backward) { return fuse_gn_ && dc_gn_fuse_pays(hw, c, 32, backward ? 1 : 0); }
  long long* gn_consumer(RB x, int c, int hw, RB x2 = RB(), int c1 = 0) {
    if (!gn_pays(hw, c, false)) return nullptr;
    long long* acc = gn_acc();
    const int cpg = c / 32;
    gn_targets_[x.p].push_back(dc_gn_target{acc, 0, 32, cpg, hw});
    if (x2.p) gn_targets_[x2.p].push_back(dc_gn_target{acc, c1, 32, cpg, hw});
    return acc;
  }
  const dc_gn_fuse* gnf(RB y) {
    if (!fuse_gn_) return nullptr;
    auto it = gn_fuse_.find(y.p);
    if (it != gn_fuse_.end()) return it->second.get();
    auto tg = gn_targets_.find(y.p);
    if (tg == gn_targets_.end()) return nullptr;
    if (tg->second.size() > 2) throw DcError(kErrArg, "GroupNorm statistics: more than two consumers");
    auto g = std::make_unique<dc_gn_fuse>();
    memset(g.get(), 0, sizeof(dc_gn_fuse));
    g->mode = 1;
    g->nt = (int)tg->second.size();
    for (int k = 0; k < g->nt; ++k) g->t[k] = tg->second[k];
    return (gn_fuse_[y.p] = std::move(g)).get();
  }
  void gn_fwd(RB x, int hw, int c, const NormW& n, bool silu, long long* acc, RB y, float* stats, RB x2 = RB(),
              int c1 = 0) {
    if (acc) ex_.groupnorm_acc(x, nb_, hw, c, n, silu, acc, y, stats, x2, c1);
    else ex_.groupnorm(x, nb_, hw, c, n, silu, y, stats, x2, c1);
  }
  // (accumulator, dc_gn_fuse mode 2) of the conv producing dL/d(GroupNorm output)
  std::pair<long long*, const dc_gn_fuse*> gn_bwd_fuse(RB x, int hw, int c, const NormW& n, bool silu,
                                                        const float* stats, RB x2 = RB(), int c1 = 0) {
    if (!gn_pays(hw, c, true)) return {nullptr, nullptr};
    long long* acc = gn_acc();
    auto g = std::make_unique<dc_gn_fuse>();
    memset(g.get(), 0, sizeof(dc_gn_fuse));
    g->mode = 2;
    g->nt = 1;
    g->t[0] = dc_gn_target{acc, 0, 32, c / 32, hw};
    g->x = x.p;
    g->ldx = x.ld;
    g->x2 = x2.p;
    g->ldx2 = x2.p ? x2.ld : 0;
    g->c1 = c1;
    g->stats = stats;
    g->gamma = n.gamma;
    g->beta = n.beta;
    g->silu = silu ? 1 : 0;
    gn_bwd_.push_back(std::move(g));
    return {acc, gn_bwd_.back().get()};
  }
  void gn_bwd(RB x, int hw, int c, const NormW& n, bool silu, const float* stats, long long* acc, RB dy, RB dx,
              RB x2 = RB(), int c1 = 0, RB add1 = RB(), RB add2 = RB()) {
    if (acc) ex_.groupnorm_bwd_acc(x, nb_, hw, c, n, stats, acc, dy, dx, x2, c1, add1, add2);
    else ex_.groupnorm_bwd(x, nb_, hw, c, n, silu, stats, dy, dx, x2, c1, add1, add2);
  }

  RB buf(long rows, int cols) { return RB(mem_.alloc((size_t)rows * cols * 2), cols); }
  float* fbuf(long n) { return (float*)mem_.alloc((size_t)n * 4); }

  RB resnet(ResnetW& r, RB x, int hh, int ww, RB x2 = RB(), int c1 = 0) {
    const int nb = nb_, P = nb * hh * ww, cin = r.cin, cout = r.cout;
    RB g1 = buf(P, cin);
    float* st1 = fbuf(nb * 32 * 2);
    RB h1 = buf(P, cout);
    float* st2 = fbuf(nb * 32 * 2);
    RB g2 = buf(P, cout);
    RB out = buf(P, cout);
    RB sc = r.has_sc ? buf(P, cout) : RB();
    ResnetW* rp = &r;
    Exec& ex = ex_;
    long long* acc1 = gn_consumer(x, cin, hh * ww, x2, c1);
    long long* acc2 = gn_consumer(h1, cout, hh * ww);
    fwd_.push_back([=, &ex]() {
      gn_fwd(x, hh * ww, cin, rp->n1, true, acc1, g1, st1, x2, c1);
      Exec::Conv a;
      a.x = g1; a.nb = nb; a.hin = hh; a.win = ww; a.cin = cin; a.hout = hh; a.wout = ww; a.cout = cout;
      a.w = rp->c1.wf; a.ktot = rp->c1.ktot_f; a.bias = rp->c1.bias; a.rowbias = rp->temb_table; a.rowbias_ld = cout;
      a.y = h1;
      conv_fwd(a);
      gn_fwd(h1, hh * ww, cout, rp->n2, true, acc2, g2, st2);
      RB res = x;
      if (rp->has_sc) {
        Exec::Conv s;
        s.x = x; s.x2 = x2; s.c1 = c1; s.nb = nb; s.hin = hh; s.win = ww; s.cin = cin; s.hout = hh; s.wout = ww;
        s.cout = cout; s.kh = 1; s.kw = 1; s.pad = 0; s.w = rp->sc.wf; s.ktot = rp->sc.ktot_f; s.bias = rp->sc.bias;
        s.y = sc;
        ex.conv(s);
        res = sc;
      }
      Exec::Conv b;
      b.x = g2; b.nb = nb; b.hin = hh; b.win = ww; b.cin = cout; b.hout = hh; b.wout = ww; b.cout = cout;
      b.w = rp->c2.wf; b.ktot = rp->c2.ktot_f; b.bias = rp->c2.bias; b.resid = res; b.y = out;
      conv_fwd(b);
    });
    TapeEntry e;
    e.kind = "resnet";
    e.r = rp;
    e.b = {{"x", x}, {"x2", x2}, {"h1", h1}, {"out", out}};
    e.f = {{"st1", st1}, {"st2", st2}};
    e.i = {{"c1", c1}, {"hh", hh}, {"ww", ww}};
    tape_.push_back(e);
    return out;
  }

  RB transformer(TransformerW& t, RB x, int hh, int ww) {
    const int nb = nb_, T = hh * ww, P = nb * T, C = t.c, H = t.heads;
    RB n0 = buf(P, C);
    float* st0 = fbuf(nb * 32 * 2);
    RB p = buf(P, C), l1 = buf(P, C);
    float* sl1 = fbuf((long)P * 2);
    RB qkv = buf(P, 3 * C), o = buf(P, C);
    float* lse = fbuf((long)nb * H * T);
    RB r1 = buf(P, C), r2 = buf(P, C);
    float* sl2 = fbuf((long)P * 2);
    float* probs = fbuf((long)P * H);
    float* sl3 = fbuf((long)P * 2);
    const dc_ln_fuse lnf3{t.ff1.csum, t.ff1.cbias, sl3};   // norm3 folded into ff.net.0.proj (unet.py ln_fuse)
    RB f8 = buf(P, 8 * C), gg = buf(P, 4 * C), out = buf(P, C);
    TransformerW* tp = &t;
    Exec& ex = ex_;
    long long* acc0 = gn_consumer(x, C, T);
    fwd_.push_back([=, &ex]() {
      gn_fwd(x, T, C, tp->norm, false, acc0, n0, st0);
      ex.linear(n0, tp->proj_in.wf, tp->proj_in.cin, P, C, p, tp->proj_in.bias);
      DCK(dc_layernorm_fwd(p.p, p.ld, P, C, tp->ln1.eps, tp->ln1.gamma, tp->ln1.beta, l1.p, l1.ld, sl1, ex.stream));
      ex.linear(l1, tp->qkv.wf, tp->qkv.cin, P, 3 * C, qkv);
      DCK(dc_attn_fwd(qkv.p, qkv.ld, nb, T, H, o.p, o.ld, lse, ex.ws, ex.ws_bytes, ex.stream));
      ex.linear(o, tp->out.wf, tp->out.cin, P, C, r1, tp->out.bias, p);
      DCK(dc_crossattn_fwd(r1.p, r1.ld, P, C, H, tp->ln2.eps, tp->ln2.gamma, tp->ln2.beta, tp->tabs, tp->c0, r2.p,
                           r2.ld, sl2, probs, sl3, tp->ln3.eps, ex.stream));
      ex.linear(r2, tp->ff1.wf, tp->ff1.cin, P, 8 * C, f8, nullptr, RB(), nullptr, 0, 1, gg, RB(), nullptr, &lnf3);
      // (FF2 + residual) -> proj_out + residual as one linear over [gg | r2] (unet.py, t.ffo)
      Exec::Conv fo = Exec::lin(gg, tp->ffo.wf, tp->ffo.cin, P, C, out, tp->ffo.bias, x);
      fo.x2 = r2;
      fo.c1 = 4 * C;
      conv_fwd(fo);
    });
    TapeEntry e;
    e.kind = "transformer";
    e.t = tp;
    e.b = {{"x", x}, {"p", p}, {"qkv", qkv}, {"o", o}, {"r1", r1}, {"r2", r2}, {"f8", f8}, {"out", out}};
    e.f = {{"st0", st0}, {"sl1", sl1}, {"lse", lse}, {"sl2", sl2}, {"probs", probs}, {"sl3", sl3}};
    e.i = {{"hh", hh}, {"ww", ww}};
    tape_.push_back(e);
    return out;
  }

  RB downsample(ConvW& cv, RB x, int hh, int ww, int* ho_, int* wo_) {
    const int nb = nb_, ho = (hh + 2 - 3) / 2 + 1, wo = (ww + 2 - 3) / 2 + 1;
    RB out = buf((long)nb * ho * wo, cv.cout);
    ConvW* c = &cv;
    Exec& ex = ex_;
    fwd_.push_back([=, &ex]() {
      Exec::Conv a;
      a.x = x; a.nb = nb; a.hin = hh; a.win = ww; a.cin = c->cin; a.hout = ho; a.wout = wo; a.cout = c->cout;
      a.stride = 2; a.w = c->wf; a.ktot = c->ktot_f; a.bias = c->bias; a.y = out;
      conv_fwd(a);
    });
    TapeEntry e;
    e.kind = "down";
    e.cv = c;
    e.b = {{"x", x}, {"out", out}};
    e.i = {{"hh", hh}, {"ww", ww}, {"ho", ho}, {"wo", wo}};
    tape_.push_back(e);
    *ho_ = ho;
    *wo_ = wo;
    return out;
  }

  RB upsample(ConvW& cv, RB x, int hh, int ww, int ho, int wo) {
    const int nb = nb_;
    RB out = buf((long)nb * ho * wo, cv.cout);
    ConvW* c = &cv;
    Exec& ex = ex_;
    fwd_.push_back([=, &ex]() {
      Exec::Conv a;
      a.x = x; a.nb = nb; a.hin = hh; a.win = ww; a.cin = c->cin; a.hout = ho; a.wout = wo; a.cout = c->cout;
      a.mode = 1; a.w = c->wf; a.ktot = c->ktot_f; a.bias = c->bias; a.y = out;
      conv_fwd(a);
    });
    TapeEntry e;
    e.kind = "up";
    e.cv = c;
    e.b = {{"x", x}, {"out", out}};
    e.i = {{"hh", hh}, {"ww", ww}, {"ho", ho}, {"wo", wo}};
    tape_.push_back(e);
    return out;
  }

  void build_forward() {
    const int nb = nb_;
    int hh = h_, ww = w_;
    const int c0 = net_.cfg.ch[0];
    RB h0 = buf((long)nb * h_ * w_, c0);
    {
      Exec& ex = ex_;
      UNetW* n = &net_;
      RB x8v = x8;
      const int H = h_, W = w_;
      fwd_.push_back([=, &ex]() {
        if (fuse_gn_) ex.memset0(gn_arena_, gn_arena_bytes_);   // every accumulator of the step starts at zero
        Exec::Conv a;
        a.x = x8v; a.nb = nb; a.hin = H; a.win = W; a.cin = 8; a.hout = H; a.wout = W; a.cout = c0;
        a.w = n->conv_in.wf; a.ktot = n->conv_in.ktot_f; a.bias = n->conv_in.bias; a.y = h0;
        a.gn = gnf(h0);
        ex.conv(a);
      });
      TapeEntry e;
      e.kind = "conv_in";
      e.b = {{"out", h0}};
      tape_.push_back(e);
    }
    struct Skip { RB t; int hh, ww; };
    std::vector<Skip> skips{{h0, hh, ww}};
    RB x = h0;
    for (auto& blk : net_.down) {
      for (size_t j = 0; j < blk.res.size(); ++j) {
        x = resnet(blk.res[j], x, hh, ww);
        if (!blk.att.empty()) x = transformer(blk.att[j], x, hh, ww);
        skips.push_back({x, hh, ww});
      }
      if (blk.has_sampler) {
        int ho, wo;
        x = downsample(blk.sampler, x, hh, ww, &ho, &wo);
        hh = ho;
        ww = wo;
        skips.push_back({x, hh, ww});
      }
    }
    x = resnet(net_.mid_res[0], x, hh, ww);
    x = transformer(net_.mid_attn, x, hh, ww);
    x = resnet(net_.mid_res[1], x, hh, ww);
    for (auto& blk : net_.up) {
      for (size_t j = 0; j < blk.res.size(); ++j) {
        Skip s = skips.back();
        skips.pop_back();
        if (s.hh != hh || s.ww != ww) throw DcError(kErrArg, "UNet skip shape mismatch");
        const int c1 = x.ld;
        x = resnet(blk.res[j], x, hh, ww, s.t, c1);
        if (!blk.att.empty()) x = transformer(blk.att[j], x, hh, ww);
      }
      if (blk.has_sampler) {
        const int ho = skips.back().hh, wo = skips.back().ww;
        x = upsample(blk.sampler, x, hh, ww, ho, wo);
        hh = ho;
        ww = wo;
      }
    }
    const int P = nb * h_ * w_;
    RB g = buf(P, c0);
    float* st = fbuf(nb * 32 * 2);
    RB xin = x;
    {
      Exec& ex = ex_;
      UNetW* n = &net_;
      RB vout = v;
      const int H = h_, W = w_;
      long long* acc_h = gn_consumer(xin, c0, H * W);
      fwd_.push_back([=, &ex]() {
        gn_fwd(xin, H * W, c0, n->norm_out, true, acc_h, g, st);
        Exec::Conv a;
        a.x = g; a.nb = nb; a.hin = H; a.win = W; a.cin = c0; a.hout = H; a.wout = W; a.cout = 4;
        a.w = n->conv_out.wf; a.ktot = n->conv_out.ktot_f; a.bias = n->conv_out.bias; a.y = vout;
        ex.conv(a);
      });
      TapeEntry e;
      e.kind = "head";
      e.b = {{"x", xin}};
      e.f = {{"st", st}};
      tape_.push_back(e);
    }
  }

  void build_backward() {
    const int nb = nb_, H = h_, W = w_;
    std::map<void*, RB> grad_of, extra_of;
    Exec& ex = ex_;
    UNetW* n = &net_;
    for (auto it = tape_.rbegin(); it != tape_.rend(); ++it) {
      TapeEntry& d = *it;
      if (d.kind == "head") {
        RB x = d.b["x"];
        const int P = nb * H * W, c0 = x.ld;
        RB dg = buf(P, c0), dx = buf(P, c0);
        grad_of[x.p] = dx;
        float* st = d.f["st"];
        RB dvv = dv;
        auto fb = gn_bwd_fuse(x, H * W, c0, n->norm_out, true, st);
        bwd_.push_back([=, &ex]() {
          Exec::Conv a;
          a.x = dvv; a.nb = nb; a.hin = H; a.win = W; a.cin = 8; a.hout = H; a.wout = W; a.cout = c0;
          a.w = n->conv_out.wd; a.ktot = n->conv_out.ktot_d; a.y = dg;
          a.gn = fb.second;
          ex.conv(a);
          gn_bwd(x, H * W, c0, n->norm_out, true, st, fb.first, dg, dx);
        });
      } else if (d.kind == "up") {
        ConvW* cv = d.cv;
        RB x = d.b["x"], out = d.b["out"];
        const int hh = d.i["hh"], ww = d.i["ww"], ho = d.i["ho"], wo = d.i["wo"];
        RB dout = grad_of.at(out.p);
        RB dhi = buf((long)nb * ho * wo, cv->cin), dx = buf((long)nb * hh * ww, cv->cin);
        grad_of[x.p] = dx;
        bwd_.push_back([=, &ex]() {
          Exec::Conv a;
          a.x = dout; a.nb = nb; a.hin = ho; a.win = wo; a.cin = cv->cout; a.hout = ho; a.wout = wo; a.cout = cv->cin;
          a.w = cv->wd; a.ktot = cv->ktot_d; a.y = dhi;
          ex.conv(a);
          DCK(dc_upsample_adjoint(dhi.p, dhi.ld, nb, ho, wo, cv->cin, hh, ww, dx.p, dx.ld, nullptr, 0, ex.stream));
        });
      } else if (d.kind == "down") {
        ConvW* cv = d.cv;
        RB x = d.b["x"], out = d.b["out"];
        const int hh = d.i["hh"], ww = d.i["ww"], ho = d.i["ho"], wo = d.i["wo"];
        RB dout = grad_of.at(out.p);
        RB dx = buf((long)nb * hh * ww, cv->cin);
        grad_of[x.p] = dx;
        auto e = extra_of.find(x.p);
        RB extra = e == extra_of.end() ? RB() : e->second;
        bwd_.push_back([=, &ex]() {
          Exec::Conv a;
          a.x = dout; a.nb = nb; a.hin = ho; a.win = wo; a.cin = cv->cout; a.hout = hh; a.wout = ww; a.cout = cv->cin;
          a.mode = 2; a.w = cv->wd; a.ktot = cv->ktot_d; a.resid = extra; a.y = dx;
          ex.conv(a);
        });
      } else if (d.kind == "transformer") {
        transformer_bwd(d, grad_of, extra_of);
      } else if (d.kind == "resnet") {
        resnet_bwd(d, grad_of, extra_of);
      } else if (d.kind == "conv_in") {
        RB out = d.b["out"];
        RB dout = grad_of.at(out.p);
        RB gxv = gx;
        bwd_.push_back([=, &ex]() {
          Exec::Conv a;
          a.x = dout; a.nb = nb; a.hin = H; a.win = W; a.cin = n->conv_in.cout; a.hout = H; a.wout = W; a.cout = 4;
          a.w = n->conv_in.wd; a.ktot = n->conv_in.ktot_d; a.y = gxv;
          ex.conv(a);
        });
      }
    }
  }

  void resnet_bwd(TapeEntry& d, std::map<void*, RB>& grad_of, std::map<void*, RB>& extra_of) {
    const int nb = nb_;
    ResnetW* r = d.r;
    RB x = d.b["x"], x2 = d.b["x2"], h1 = d.b["h1"], out = d.b["out"];
    const int c1 = d.i["c1"], hh = d.i["hh"], ww = d.i["ww"];
    float *st1 = d.f["st1"], *st2 = d.f["st2"];
    const int P = nb * hh * ww, cin = r->cin, cout = r->cout;
    RB dout = grad_of.at(out.p);
    RB dg2 = buf(P, cout), dh1 = buf(P, cout), dg1 = buf(P, cin), dx = buf(P, cin);
    RB extra;
    if (x2.p) {
      grad_of[x.p] = dx;
      extra_of[x2.p] = dx.col(c1);
    } else {
      grad_of[x.p] = dx;
      auto e = extra_of.find(x.p);
      if (e != extra_of.end()) extra = e->second;
    }
    Exec& ex = ex_;
    auto f2 = gn_bwd_fuse(h1, hh * ww, cout, r->n2, true, st2);
    auto f1 = gn_bwd_fuse(x, hh * ww, cin, r->n1, true, st1, x2, c1);
    // the shortcut's input-gradient into its own buffer, added by the GroupNorm backward (as unet.py, which runs it
    // as a concurrent graph branch)
    RB dsc = r->has_sc ? buf(P, cin) : RB();
    bwd_.push_back([=, &ex]() {
      if (r->has_sc) {
        Exec::Conv s;
        s.x = dout; s.nb = nb; s.hin = hh; s.win = ww; s.cin = cout; s.hout = hh; s.wout = ww; s.cout = cin;
        s.kh = 1; s.kw = 1; s.pad = 0; s.w = r->sc.wd; s.ktot = r->sc.ktot_d; s.y = dsc;
        ex.conv(s);
      }
      Exec::Conv a;
      a.x = dout; a.nb = nb; a.hin = hh; a.win = ww; a.cin = cout; a.hout = hh; a.wout = ww; a.cout = cout;
      a.w = r->c2.wd; a.ktot = r->c2.ktot_d; a.y = dg2;
      a.gn = f2.second;
      ex.conv(a);
      gn_bwd(h1, hh * ww, cout, r->n2, true, st2, f2.first, dg2, dh1);
      Exec::Conv b;
      b.x = dh1; b.nb = nb; b.hin = hh; b.win = ww; b.cin = cout; b.hout = hh; b.wout = ww; b.cout = cin;
      b.w = r->c1.wd; b.ktot = r->c1.ktot_d; b.y = dg1;
      b.gn = f1.second;
      ex.conv(b);
      gn_bwd(x, hh * ww, cin, r->n1, true, st1, f1.first, dg1, dx, x2, c1, r->has_sc ? dsc : dout, extra);
    });
  }

  void transformer_bwd(TapeEntry& d, std::map<void*, RB>& grad_of, std::map<void*, RB>& extra_of) {
    const int nb = nb_;
    TransformerW* t = d.t;
    RB x = d.b["x"];
    const int hh = d.i["hh"], ww = d.i["ww"], T = hh * ww, P = nb * T, C = t->c, H = t->heads;
    RB out = d.b["out"];
    RB dout = grad_of.at(out.p);
    RB dr3 = buf(P, C), df = buf(P, 8 * C), dl3 = buf(P, C), dr1 = buf(P, C), dob = buf(P, C),
       dqkv = buf(P, 3 * C), dl1 = buf(P, C), dp = buf(P, C), dn0 = buf(P, C), dx = buf(P, C);
    float* delta = fbuf(2L * nb * H * T);   // dc_attn_bwd's row constants (-delta, -8 lse)
    grad_of[x.p] = dx;
    auto e = extra_of.find(x.p);
    RB extra = e == extra_of.end() ? RB() : e->second;
    RB p = d.b["p"], qkv = d.b["qkv"], o = d.b["o"], r1 = d.b["r1"], r2 = d.b["r2"], f8 = d.b["f8"];
    float *st0 = d.f["st0"], *sl1 = d.f["sl1"], *lse = d.f["lse"], *sl2 = d.f["sl2"], *probs = d.f["probs"],
          *sl3 = d.f["sl3"];
    Exec& ex = ex_;
    auto f0 = gn_bwd_fuse(x, T, C, t->norm, false, st0);
    bwd_.push_back([=, &ex]() {
      // dL/dgg (+ GEGLU backward) into df and dL/dr2 into dr3 from the folded linear's input-gradient (unet.py)
      Exec::Conv fb = Exec::lin(dout, t->ffo.wd, C, P, 5 * C, df, nullptr, RB(), nullptr, 0, 2, dr3, f8);
      fb.geglu_n = 4 * C;
      ex.conv(fb);
      ex.linear(df, t->ff1.wd, t->ff1.cout, P, C, dl3);
      // norm3 backward inside the cross-attention backward (dl3 = gamma3 dL/dLN3 through the folded weight)
      DCK(dc_crossattn_bwd_ln(r1.p, r1.ld, P, C, H, t->ln2.gamma, t->tabs, sl2, probs, dl3.p, dl3.ld, r2.p, r2.ld, sl3,
                              dr3.p, dr3.ld, dr1.p, dr1.ld, ex.stream));
      ex.linear(dr1, t->out.wd, t->out.cout, P, C, dob);
      DCK(dc_attn_bwd(qkv.p, qkv.ld, o.p, o.ld, dob.p, dob.ld, lse, nb, T, H, delta, dqkv.p, dqkv.ld, ex.ws,
                      ex.ws_bytes, ex.stream));
      ex.linear(dqkv, t->qkv.wd, t->qkv.cout, P, C, dl1);
      DCK(dc_layernorm_bwd(p.p, p.ld, P, C, t->ln1.gamma, sl1, dl1.p, dl1.ld, dp.p, dp.ld, dr1.p, dr1.ld,
                           ex.stream));
      ex.linear(dp, t->proj_in.wd, t->proj_in.cout, P, C, dn0, nullptr, RB(), nullptr, 0, 0, RB(), RB(), f0.second);
      gn_bwd(x, T, C, t->norm, false, st0, f0.first, dn0, dx, RB(), 0, dout, extra);
    });
  }
};

// ------------------------------------------------------------------ TAESD (taesd.py)
constexpr int kCH = 64;
const int kDecBlocks[4] = {3, 3, 3, 1};
const int kEncBlocks[4] = {1, 3, 3, 3};

struct TAESDW {
  ConvW dec_in, dec_out, enc_out;
  struct Item { bool block; ConvW c[3]; ConvW up; };
  std::vector<Item> dec;
  struct EncItem { int kind; ConvW c[3]; };  // 0 conv, 1 down, 2 block
  std::vector<EncItem> enc;
};

void load_taesd(TAESDW& t, Loader& L) {
  const std::vector<int> in_rows{0, 1, 2, 3};
  t.dec_in = L.conv("decoder.layers.0", true, 1, 8, true, &in_rows);
  int i = 2;
  for (int bi = 0; bi < 4; ++bi) {
    for (int k = 0; k < kDecBlocks[bi]; ++k) {
      TAESDW::Item it;
      it.block = true;
      for (int c = 0; c < 3; ++c)
        it.c[c] = L.conv("decoder.layers." + std::to_string(i) + ".conv." + std::to_string(2 * c), true);
      t.dec.push_back(it);
      ++i;
    }
    if (bi < 3) {
      ++i;  // nn.Upsample
      TAESDW::Item it;
      it.block = false;
      it.up = L.conv("decoder.layers." + std::to_string(i), false);
      t.dec.push_back(it);
      ++i;
    }
  }
  t.dec_out = L.conv("decoder.layers." + std::to_string(i), true, 1, 0, true, nullptr, 8);
  i = 0;
  for (int bi = 0; bi < 4; ++bi) {
    TAESDW::EncItem e;
    if (bi == 0) {
      e.kind = 0;
      e.c[0] = L.conv("encoder.layers." + std::to_string(i), true, 1, 8, false);
    } else {
      e.kind = 1;
      e.c[0] = L.conv("encoder.layers." + std::to_string(i), false, 2, 0, false);
    }
    t.enc.push_back(e);
    ++i;
    for (int k = 0; k < kEncBlocks[bi]; ++k) {
      TAESDW::EncItem b;
      b.kind = 2;
      for (int c = 0; c < 3; ++c)
        b.c[c] = L.conv("encoder.layers." + std::to_string(i) + ".conv." + std::to_string(2 * c), true, 1, 0, false);
      t.enc.push_back(b);
      ++i;
    }
  }
  t.enc_out = L.conv("encoder.layers." + std::to_string(i), true, 1, 0, false);
}

// TAESDHIP.encode: img8 [nb*H*W][8] -> 4 latent channels into `out`
void taesd_encode(TAESDW& t, Exec& ex, DevMem& scratch, RB img8, int nb, int H, int W, RB out) {
  int hh = H, ww = W;
  RB x = img8;
  auto conv = [&](RB in, const ConvW& c, int cin, int hin, int win, int hout, int wout, int cout, int stride, RB y,
                  RB resid, int act) {
    Exec::Conv a;
    a.x = in; a.nb = nb; a.hin = hin; a.win = win; a.cin = cin; a.hout = hout; a.wout = wout; a.cout = cout;
    a.stride = stride; a.w = c.wf; a.ktot = c.ktot_f; a.bias = c.bias; a.resid = resid; a.act = act; a.y = y;
    ex.conv(a);
  };
  for (auto& e : t.enc) {
    if (e.kind == 0) {
      RB y((void*)scratch.alloc((size_t)nb * hh * ww * kCH * 2, false), kCH);
      conv(x, e.c[0], 8, hh, ww, hh, ww, kCH, 1, y, RB(), 0);
      x = y;
    } else if (e.kind == 1) {
      const int ho = (hh - 1) / 2 + 1, wo = (ww - 1) / 2 + 1;
      RB y((void*)scratch.alloc((size_t)nb * ho * wo * kCH * 2, false), kCH);
      conv(x, e.c[0], kCH, hh, ww, ho, wo, kCH, 2, y, RB(), 0);
      hh = ho;
      ww = wo;
      x = y;
    } else {
      const size_t P = (size_t)nb * hh * ww;
      RB a1(scratch.alloc(P * kCH * 2, false), kCH), a2(scratch.alloc(P * kCH * 2, false), kCH),
          o(scratch.alloc(P * kCH * 2, false), kCH);
      conv(x, e.c[0], kCH, hh, ww, hh, ww, kCH, 1, a1, RB(), 1);
      conv(a1, e.c[1], kCH, hh, ww, hh, ww, kCH, 1, a2, RB(), 1);
      conv(a2, e.c[2], kCH, hh, ww, hh, ww, kCH, 1, o, x, 1);
      x = o;
    }
  }
  conv(x, t.enc_out, kCH, hh, ww, hh, ww, 4, 1, out, RB(), 0);
}

// sparse-aware decode row sets: (row list, padded count) for the launches named out, c3, c2, c1, up, dhi
struct RowSets {
  std::pair<const int*, int> s[6];
};
enum { kOut = 0, kC3, kC2, kC1, kUp, kDhi };

class DecoderPlan {
 public:
  DecoderPlan(TAESDW& net, Exec& ex, DevMem& mem, int nb, int h, int w) : net_(net), ex_(ex), mem_(mem), nb_(nb) {
    tin = buf((long)nb * h * w, 8);
    dtin = buf((long)nb * h * w, 8);
    int hh = h, ww = w;
    RB a0 = buf((long)nb * hh * ww, kCH);
    Exec& exr = ex_;
    TAESDW* n = &net_;
    const RowSets* const* rows = &rows_;
    {
      RB tinv = tin;
      fwd_.push_back([=, &exr]() {
        Exec::Conv a;
        a.x = tinv; a.nb = nb; a.hin = hh; a.win = ww; a.cin = 8; a.hout = hh; a.wout = ww; a.cout = kCH;
        a.w = n->dec_in.wf; a.ktot = n->dec_in.ktot_f; a.bias = n->dec_in.bias; a.act = 1; a.y = a0;
        exr.conv(a);
      });
    }
    struct Tp { bool block; TAESDW::Item* it; RB x; bool xr; RB a1, a2, o, y; int hh, ww, ho, wo; };
    std::vector<Tp> tape;
    RB x = a0;
    bool x_relu = true;
    // the full-resolution size is known only after the loop: compute it first
    int fh = h, fw = w;
    for (auto& it : net_.dec) if (!it.block) { fh *= 2; fw *= 2; }
    H_ = fh;
    W_ = fw;
    for (auto& it : net_.dec) {
      const long P = (long)nb * hh * ww;
      if (it.block) {
        RB a1 = buf(P, kCH), a2 = buf(P, kCH), o = buf(P, kCH);
        const bool full = (hh == fh && ww == fw);
        TAESDW::Item* ip = &it;
        fwd_.push_back([=, &exr]() {
          const RowSets* rs = *rows;
          auto R = [&](int k) { return (rs && full) ? rs->s[k] : std::pair<const int*, int>(nullptr, 0); };
          Exec::Conv a;
          a.nb = nb; a.hin = hh; a.win = ww; a.cin = kCH; a.hout = hh; a.wout = ww; a.cout = kCH; a.act = 1;
          a.x = x; a.w = ip->c[0].wf; a.ktot = ip->c[0].ktot_f; a.bias = ip->c[0].bias; a.y = a1;
          a.rows = R(kC1).first; a.nrows = R(kC1).second;
          exr.conv(a);
          a.x = a1; a.w = ip->c[1].wf; a.ktot = ip->c[1].ktot_f; a.bias = ip->c[1].bias; a.y = a2;
          a.rows = R(kC2).first; a.nrows = R(kC2).second;
          exr.conv(a);
          a.x = a2; a.w = ip->c[2].wf; a.ktot = ip->c[2].ktot_f; a.bias = ip->c[2].bias; a.resid = x; a.y = o;
          a.rows = R(kC3).first; a.nrows = R(kC3).second;
          exr.conv(a);
        });
        tape.push_back({true, ip, x, x_relu, a1, a2, o, RB(), hh, ww, 0, 0});
        x = o;
        x_relu = true;
      } else {
        const int ho = 2 * hh, wo = 2 * ww;
        RB y = buf((long)nb * ho * wo, kCH);
        const bool full = (ho == fh && wo == fw);
        TAESDW::Item* ip = &it;
        fwd_.push_back([=, &exr]() {
          const RowSets* rs = *rows;
          Exec::Conv a;
          a.x = x; a.nb = nb; a.hin = hh; a.win = ww; a.cin = kCH; a.hout = ho; a.wout = wo; a.cout = kCH; a.mode = 1;
          a.w = ip->up.wf; a.ktot = ip->up.ktot_f; a.y = y;
          if (rs && full) { a.rows = rs->s[kUp].first; a.nrows = rs->s[kUp].second; }
          exr.conv(a);
        });
        tape.push_back({false, ip, x, x_relu, RB(), RB(), RB(), y, hh, ww, ho, wo});
        x = y;
        x_relu = false;
        hh = ho;
        ww = wo;
      }
    }
    out = buf((long)nb * hh * ww, 8);
    dout = buf((long)nb * hh * ww, 8);
    RB xl = x;
    {
      RB outv = out;
      fwd_.push_back([=, &exr]() {
        const RowSets* rs = *rows;
        Exec::Conv a;
        a.x = xl; a.nb = nb; a.hin = hh; a.win = ww; a.cin = kCH; a.hout = hh; a.wout = ww; a.cout = 3;
        a.w = n->dec_out.wf; a.ktot = n->dec_out.ktot_f; a.bias = n->dec_out.bias; a.y = outv;
        if (rs) { a.rows = rs->s[kOut].first; a.nrows = rs->s[kOut].second; }
        exr.conv(a);
      });
    }
    // backward
    const long P = (long)nb * hh * ww;
    RB dpre = buf(P, kCH);
    full_res_grads_.push_back(dpre);
    const bool last_relu = x_relu;
    {
      RB doutv = dout;
      bwd_.push_back([=, &exr]() {
        const RowSets* rs = *rows;
        Exec::Conv a;
        a.x = doutv; a.nb = nb; a.hin = hh; a.win = ww; a.cin = 8; a.hout = hh; a.wout = ww; a.cout = kCH;
        a.w = n->dec_out.wd; a.ktot = n->dec_out.ktot_d; a.mask = last_relu ? xl : RB(); a.y = dpre;
        if (rs) { a.rows = rs->s[kC3].first; a.nrows = rs->s[kC3].second; }
        exr.conv(a);
      });
    }
    RB g = dpre;
    for (auto it = tape.rbegin(); it != tape.rend(); ++it) {
      const Tp d = *it;
      if (d.block) {
        const long Pb = (long)nb * d.hh * d.ww;
        RB dc2 = buf(Pb, kCH), dc1 = buf(Pb, kCH), dx = buf(Pb, kCH);
        const bool full = (d.hh == fh && d.ww == fw);
        if (full) { full_res_grads_.push_back(dc2); full_res_grads_.push_back(dc1); full_res_grads_.push_back(dx); }
        const RB gg = g;
        bwd_.push_back([=, &exr]() {
          const RowSets* rs = *rows;
          auto R = [&](int k) { return (rs && full) ? rs->s[k] : std::pair<const int*, int>(nullptr, 0); };
          Exec::Conv a;
          a.nb = nb; a.hin = d.hh; a.win = d.ww; a.cin = kCH; a.hout = d.hh; a.wout = d.ww; a.cout = kCH;
          a.x = gg; a.w = d.it->c[2].wd; a.ktot = d.it->c[2].ktot_d; a.mask = d.a2; a.y = dc2;
          a.rows = R(kC2).first; a.nrows = R(kC2).second;
          exr.conv(a);
          a.x = dc2; a.w = d.it->c[1].wd; a.ktot = d.it->c[1].ktot_d; a.mask = d.a1; a.y = dc1;
          a.rows = R(kC1).first; a.nrows = R(kC1).second;
          exr.conv(a);
          a.x = dc1; a.w = d.it->c[0].wd; a.ktot = d.it->c[0].ktot_d; a.resid = gg; a.mask = d.xr ? d.x : RB(); a.y = dx;
          a.rows = R(kUp).first; a.nrows = R(kUp).second;
          exr.conv(a);
        });
        g = dx;
      } else {
        RB dhi = buf((long)nb * d.ho * d.wo, kCH), dlo = buf((long)nb * d.hh * d.ww, kCH);
        const bool full = (d.ho == fh && d.wo == fw);
        if (full) full_res_grads_.push_back(dhi);
        const RB gg = g;
        bwd_.push_back([=, &exr]() {
          const RowSets* rs = *rows;
          Exec::Conv a;
          a.x = gg; a.nb = nb; a.hin = d.ho; a.win = d.wo; a.cin = kCH; a.hout = d.ho; a.wout = d.wo; a.cout = kCH;
          a.w = d.it->up.wd; a.ktot = d.it->up.ktot_d; a.y = dhi;
          if (rs && full) { a.rows = rs->s[kDhi].first; a.nrows = rs->s[kDhi].second; }
          exr.conv(a);
          DCK(dc_upsample_adjoint(dhi.p, dhi.ld, nb, d.ho, d.wo, kCH, d.hh, d.ww, dlo.p, dlo.ld,
                                  d.xr ? d.x.p : nullptr, d.xr ? d.x.ld : 0, exr.stream));
        });
        g = dlo;
      }
    }
    {
      const RB g0 = g;
      RB dtinv = dtin;
      bwd_.push_back([=, &exr]() {
        Exec::Conv a;
        a.x = g0; a.nb = nb; a.hin = h; a.win = w; a.cin = kCH; a.hout = h; a.wout = w; a.cout = 4;
        a.w = n->dec_in.wd; a.ktot = n->dec_in.ktot_d; a.y = dtinv;
        exr.conv(a);
      });
    }
  }
  // taesd.DecoderPlan.set_rows
  void set_rows(const RowSets* rs) {
    rows_ = rs;
    if (rs)
      for (const RB& t : full_res_grads_) ex_.memset0(t.p, (size_t)nb_ * H_ * W_ * kCH * 2);
  }
  void forward() { for (auto& f : fwd_) f(); }
  void backward() { for (auto& f : bwd_) f(); }
  RB tin, dtin, out, dout;
  int H_ = 0, W_ = 0;

 private:
  TAESDW& net_;
  Exec& ex_;
  DevMem& mem_;
  int nb_;
  const RowSets* rows_ = nullptr;
  std::vector<RB> full_res_grads_;
  std::vector<std::function<void()>> fwd_, bwd_;
  RB buf(long rows, int cols) { return RB(mem_.alloc((size_t)rows * cols * 2), cols); }
};

// ------------------------------------------------------------------ per-(frames, h, w) state (pipeline._plan)
struct PlanState {
  std::unique_ptr<UNetPlan> unet;
  std::unique_ptr<DecoderPlan> dec;
  DevMem mem;
  RB x0, gdir;
  float *eps_norm, *affine, *m_aff, *v_aff, *daff, *loss, *dbg, *dA;
  void *m_lat, *v_lat;
  int n = 0, h = 0, w = 0;
  // per-call tables bound by the captured graph (refreshed in place on replay)
  int tab_hw = 0, tab_steps = 0;
  float *coef = nullptr, *adam = nullptr, *gval = nullptr, *params = nullptr;
  int *idx = nullptr, *cnt = nullptr;
  DevMem tabs;
  // sparse-aware decode row sets
  long rs_total = 0;
  unsigned char* masks = nullptr;
  int *lists = nullptr, *rs_ws = nullptr, *rs_cnt = nullptr;
  DevMem rsmem;
  RowSets rowsets;
  bool have_rows = false;
  // captured step
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  std::vector<double> gkey;
  ~PlanState() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

}  // namespace

// ------------------------------------------------------------------ session
struct dc_session {
  int device = 0;
  hipStream_t stream = nullptr;  // the session's own launch stream (graphs capture on it)
  DevMem wmem;                   // weights
  DevMem cmem;                   // ctx workspace / step counter
  Exec ex;
  UNetW unet;
  TAESDW taesd;
  bool loaded = false;
  std::map<std::tuple<int, int, int>, std::unique_ptr<PlanState>> plans;
  std::string err;
  bool sparse_decode = true;
};

namespace {

void timestep_tables(dc_session* s, PlanState& st, int steps, const long long* ts) {
  // UNetHIP.build_temb_tables: t_emb (fp32, host) -> bf16 -> linear_1 -> SiLU -> linear_2 -> SiLU -> per-resnet
  // time_emb_proj, all on the device
  const int c0 = s->unet.cfg.ch[0], d = s->unet.t_lin1.cout;
  std::vector<float> te((size_t)steps * c0);
  DCK(dc_timestep_embedding(ts, steps, c0, te.data()));
  std::vector<uint16_t> teb = to_bf16(te);
  Exec& ex = s->ex;
  DevMem tmp;   // freed after the stream drains (end of this function)
  void* teh = tmp.alloc(teb.size() * 2, false);
  HIPK(hipMemcpyAsync(teh, teb.data(), teb.size() * 2, hipMemcpyHostToDevice, s->stream));
  HIPK(hipStreamSynchronize(s->stream));
  RB h1(tmp.alloc((size_t)steps * d * 2), d), a1(tmp.alloc((size_t)steps * d * 2), d),
      emb(tmp.alloc((size_t)steps * d * 2), d), semb(tmp.alloc((size_t)steps * d * 2), d);
  ex.linear(RB(teh, c0), s->unet.t_lin1.wf, c0, steps, d, h1, s->unet.t_lin1.bias);
  DCK(dc_silu(h1.p, (long long)steps * d, a1.p, ex.stream));
  ex.linear(a1, s->unet.t_lin2.wf, d, steps, d, emb, s->unet.t_lin2.bias);
  DCK(dc_silu(emb.p, (long long)steps * d, semb.p, ex.stream));
  for (ResnetW* r : s->unet.resnets()) {
    auto it = r->temb_tables.find(steps);
    if (it == r->temb_tables.end())
      it = r->temb_tables.emplace(steps, s->wmem.alloc((size_t)steps * r->cout * 2, false)).first;
    r->temb_table = it->second;
    ex.linear(semb, r->temb.wf, d, steps, r->cout, RB(r->temb_table, r->cout), r->temb.bias);
  }
  HIPK(hipStreamSynchronize(s->stream));
}

PlanState& plan(dc_session* s, int n, int h, int w) {
  auto key = std::make_tuple(n, h, w);
  auto it = s->plans.find(key);
  if (it != s->plans.end()) return *it->second;
  auto st = std::make_unique<PlanState>();
  st->n = n;
  st->h = h;
  st->w = w;
  st->unet = std::make_unique<UNetPlan>(s->unet, s->ex, st->mem, n, h, w);
  st->dec = std::make_unique<DecoderPlan>(s->taesd, s->ex, st->mem, n, h, w);
  const long P = (long)n * h * w;
  st->x0 = RB(st->mem.alloc(P * 8 * 2), 8);
  st->gdir = RB(st->mem.alloc(P * 8 * 2), 8);
  st->eps_norm = (float*)st->mem.alloc(n * 4);
  st->m_lat = st->mem.alloc(P * 4 * 2);
  st->v_lat = st->mem.alloc(P * 4 * 2);
  st->affine = (float*)st->mem.alloc(n * 2 * 4);
  st->m_aff = (float*)st->mem.alloc(n * 2 * 4);
  st->v_aff = (float*)st->mem.alloc(n * 2 * 4);
  st->daff = (float*)st->mem.alloc(n * 2 * 4);
  st->loss = (float*)st->mem.alloc(n * 4);
  st->dbg = (float*)st->mem.alloc(n * 4 * 4);
  st->dA = (float*)st->mem.alloc((size_t)n * st->dec->H_ * st->dec->W_ * 4);
  PlanState& ref = *st;
  s->plans.emplace(key, std::move(st));
  return ref;
}

struct Geo {
  int n, H, W, RH, RW, PH, PW, h, w;
};

Geo geometry(int n, int H, int W, int res) {
  Geo g;
  g.n = n; g.H = H; g.W = W;
  const int m = std::max(H, W);
  g.RH = H * res / m;
  g.RW = W * res / m;
  g.PH = (g.RH + 7) / 8 * 8;
  g.PW = (g.RW + 7) / 8 * 8;
  g.h = g.PH / 8;
  g.w = g.PW / 8;
  return g;
}

void check_params(const dc_sample_params* p) {
  if (!p) throw DcError(kErrArg, "params is null");
  if (p->norm != 0 && p->norm != 1)
    throw DcError(kErrArg, "norm must be const (0) or minmax (1) in the native session (percentile: Python host)");
  if (p->projection < 0 || p->projection > 2) throw DcError(kErrArg, "Unknown projection method");
  if ((p->projection != 0 || p->inv) && p->min_depth <= 1e-7f)
    throw DcError(kErrArg, "min_depth must be > 1e-07 when projection is 'log' or 'log10' or inv is True");
  if (!(p->beta > 0.0f && p->beta < 1.0f)) throw DcError(kErrArg, "beta must be in (0, 1)");
  if (p->steps <= 0 || p->resolution <= 0) throw DcError(kErrArg, "steps and resolution must be > 0");
  if (p->opt < 0 || p->opt > 2) throw DcError(kErrArg, "Unknown optimizer");
  if (p->interp < 0 || p->interp > 1) throw DcError(kErrArg, "Unknown interp_mode");
}

// pipeline._decode_rows: the six row sets, or none (dense decode) when the largest covers most of the map
bool decode_rows(dc_session* s, PlanState& st, const Geo& g) {
  const long total = (long)g.n * g.PH * g.PW;
  if (st.rs_total != total) {
    st.rsmem = DevMem();
    st.masks = (unsigned char*)st.rsmem.alloc((size_t)6 * total, false);
    st.lists = (int*)st.rsmem.alloc((size_t)6 * total * 4, false);
    st.rs_ws = (int*)st.rsmem.alloc((size_t)dc_mask_rows_ws_bytes(total) + 16, false);
    st.rs_cnt = (int*)st.rsmem.alloc(6 * 4);
    st.rs_total = total;
  }
  hipStream_t hs = s->stream;
  DCK(dc_tap_mask(st.idx, st.cnt, st.params, g.n, g.PH, g.PW, g.RH, g.RW, g.H, g.W, st.masks, hs));
  for (int k = 1; k < 6; ++k) DCK(dc_dilate_mask(st.masks + (size_t)(k - 1) * total, g.n, g.PH, g.PW, st.masks + (size_t)k * total, hs));
  for (int k = 0; k < 6; ++k) {
    DCK(dc_mask_count(st.masks + (size_t)k * total, total, st.rs_ws, st.rs_cnt + k, hs));
    int c = 0;
    HIPK(hipMemcpyAsync(&c, st.rs_cnt + k, 4, hipMemcpyDeviceToHost, hs));
    HIPK(hipStreamSynchronize(hs));
    if (k == 5 && c > 0.6 * total) return false;
    const long cm = std::max(c - 1, 1);
    int bl = 0;
    while ((1L << bl) <= cm) ++bl;   // int.bit_length()
    const long gran = std::max(4096L, (1L << bl) / 4);
    const long pad = std::min(total, (std::max((long)c, 1L) + gran - 1) / gran * gran);
    DCK(dc_mask_rows(st.masks + (size_t)k * total, total, st.rs_ws, st.rs_cnt + k, (int)pad, st.lists + (size_t)k * total, hs));
    st.rowsets.s[k] = {st.lists + (size_t)k * total, (int)pad};
  }
  return true;
}

// pipeline.MarigoldDepthCompletionPipeline._step
void guided_step(dc_session* s, PlanState& st, const Geo& g, int steps, int opt) {
  Exec& ex = s->ex;
  UNetPlan& up = *st.unet;
  DecoderPlan& dp = *st.dec;
  hipStream_t hs = ex.stream;
  const int n = g.n, hw = g.h * g.w;
  const long P = (long)n * hw;
  up.forward();
  DCK(dc_preview(up.x8.p, up.v.p, n, hw, st.coef, ex.step, st.x0.p, dp.tin.p, st.eps_norm, hs));
  dp.forward();
  ex.memset0(st.dA, (size_t)n * dp.H_ * dp.W_ * 4);
  DCK(dc_sparse_loss(dp.out.p, 8, n, g.PH, g.PW, g.RH, g.RW, g.H, g.W, st.idx, st.gval, st.cnt, st.params, st.affine,
                     st.dA, st.daff, st.loss, hs));
  DCK(dc_decode_tail_bwd(dp.out.p, 8, st.dA, n, g.PH, g.PW, g.RH, g.RW, dp.dout.p, hs));
  dp.backward();
  DCK(dc_taesd_clamp_bwd(st.x0.p, 8, dp.dtin.p, 8, P, st.coef, ex.step, st.gdir.p, up.dv.p, hs));
  up.backward();
  DCK(dc_latent_update(up.x8.p, up.v.p, st.gdir.p, up.gx.p, n, hw, st.coef, st.adam, ex.step, st.eps_norm, st.m_lat,
                       st.v_lat, st.affine, st.m_aff, st.v_aff, st.daff, st.dbg, opt, 0, 0.1f, ex.ws, ex.ws_bytes, hs));
  DCK(dc_step_advance(ex.step, steps, hs));
}

void reset_state(dc_session* s, PlanState& st, const Geo& g, const void* noise, int noise_n, const void* prev,
                 float beta) {
  Exec& ex = s->ex;
  DCK(dc_latent_init(noise, noise_n, prev, beta, g.n, g.h * g.w, st.unet->x8.p, ex.stream));
  const long P = (long)g.n * g.h * g.w;
  ex.memset0(st.m_lat, P * 4 * 2);
  ex.memset0(st.v_lat, P * 4 * 2);
  ex.memset0(st.m_aff, g.n * 2 * 4);
  ex.memset0(st.v_aff, g.n * 2 * 4);
  std::vector<float> aff((size_t)g.n * 2);
  for (int i = 0; i < g.n; ++i) { aff[2 * i] = 1.0f; aff[2 * i + 1] = 0.0f; }
  HIPK(hipMemcpyAsync(st.affine, aff.data(), aff.size() * 4, hipMemcpyHostToDevice, ex.stream));
  HIPK(hipStreamSynchronize(ex.stream));
  ex.memset0(ex.step, 4);
}

// __call__ from the latent init to the end of the denoising loop; img latents already in x8[..., 0:4]
void sample(dc_session* s, PlanState& st, const Geo& g, const void* noise, int noise_n, const void* prev,
            const float* sparses, const dc_sample_params* p) {
  Exec& ex = s->ex;
  hipStream_t hs = ex.stream;
  const int n = g.n;
  const long HWs = (long)g.H * g.W;
  // per-call tables: sized by the call; a size change drops the captured graph (it binds these addresses)
  if (st.tab_hw != HWs || st.tab_steps != p->steps) {
    if (st.gexec) { (void)hipGraphExecDestroy(st.gexec); st.gexec = nullptr; }
    if (st.graph) { (void)hipGraphDestroy(st.graph); st.graph = nullptr; }
    st.gkey.clear();
    st.tabs = DevMem();
    st.idx = (int*)st.tabs.alloc((size_t)n * HWs * 4, false);
    st.gval = (float*)st.tabs.alloc((size_t)n * HWs * 4, false);
    st.cnt = (int*)st.tabs.alloc(n * 4, false);
    st.params = (float*)st.tabs.alloc(n * 8 * 4, false);
    st.coef = (float*)st.tabs.alloc((size_t)p->steps * 4 * 4, false);
    st.adam = (float*)st.tabs.alloc((size_t)p->steps * 4 * 4, false);
    st.tab_hw = (int)HWs;
    st.tab_steps = p->steps;
  }
  DCK(dc_latent_init(noise, noise_n, prev, p->beta, n, g.h * g.w, st.unet->x8.p, hs));
  // sparse guides (marigold_dc.py:706-756)
  DCK(dc_sparse_setup(sparses, n, g.H, g.W, p->norm, p->min_depth, p->max_depth, nullptr, p->projection, p->inv,
                      p->interp, st.idx, st.gval, st.cnt, st.params, hs));
  std::vector<int> cnt_h(n);
  HIPK(hipMemcpyAsync(cnt_h.data(), st.cnt, n * 4, hipMemcpyDeviceToHost, hs));
  HIPK(hipStreamSynchronize(hs));
  for (int c : cnt_h)
    if (c == 0)
      throw DcError(kErrArg, "No valid values found in mask for some positions. Ensure that mask has at least one "
                             "True value along the specified dimensions.");
  // sparse-aware decode
  st.have_rows = s->sparse_decode && decode_rows(s, st, g);
  st.dec->set_rows(st.have_rows ? &st.rowsets : nullptr);
  // tables (DDIMTables.coef, adam_table) and the per-resnet time embeddings
  std::vector<long long> ts(p->steps);
  std::vector<float> coef((size_t)p->steps * 4), adam((size_t)p->steps * 4);
  DCK(dc_schedule_tables(p->steps, p->lr_latent, p->lr_scaling, p->opt, ts.data(), coef.data(), adam.data()));
  HIPK(hipMemcpyAsync(st.coef, coef.data(), coef.size() * 4, hipMemcpyHostToDevice, hs));
  HIPK(hipMemcpyAsync(st.adam, adam.data(), adam.size() * 4, hipMemcpyHostToDevice, hs));
  HIPK(hipStreamSynchronize(hs));
  timestep_tables(s, st, p->steps, ts.data());
  const long P = (long)n * g.h * g.w;
  ex.memset0(st.m_lat, P * 4 * 2);
  ex.memset0(st.v_lat, P * 4 * 2);
  ex.memset0(st.m_aff, n * 2 * 4);
  ex.memset0(st.v_aff, n * 2 * 4);
  ex.memset0(st.daff, n * 2 * 4);
  std::vector<float> aff((size_t)n * 2);
  for (int i = 0; i < n; ++i) { aff[2 * i] = 1.0f; aff[2 * i + 1] = 0.0f; }
  HIPK(hipMemcpyAsync(st.affine, aff.data(), aff.size() * 4, hipMemcpyHostToDevice, hs));
  HIPK(hipStreamSynchronize(hs));
  ex.memset0(ex.step, 4);
  // denoising loop: one captured step replayed `steps` times (the graph is re-captured when its key changes)
  if (p->use_graph) {
    std::vector<double> key{(double)p->steps, (double)g.H, (double)g.W, (double)g.RH, (double)g.RW, p->lr_latent,
                            p->lr_scaling, (double)p->opt, st.have_rows ? 1.0 : 0.0};
    if (st.have_rows)
      for (int k = 0; k < 6; ++k) key.push_back(st.rowsets.s[k].second);
    if (!st.gexec || key != st.gkey) {
      if (st.gexec) { (void)hipGraphExecDestroy(st.gexec); st.gexec = nullptr; }
      if (st.graph) { (void)hipGraphDestroy(st.graph); st.graph = nullptr; }
      guided_step(s, st, g, p->steps, p->opt);  // warm-up (first-use lazy initialisation), then undo its effect
      HIPK(hipStreamSynchronize(hs));
      reset_state(s, st, g, noise, noise_n, prev, p->beta);
      HIPK(hipStreamBeginCapture(hs, hipStreamCaptureModeThreadLocal));
      try {
        guided_step(s, st, g, p->steps, p->opt);
      } catch (...) {
        hipGraph_t junk;
        (void)hipStreamEndCapture(hs, &junk);
        if (junk) (void)hipGraphDestroy(junk);
        throw;
      }
      HIPK(hipStreamEndCapture(hs, &st.graph));
      HIPK(hipGraphInstantiate(&st.gexec, st.graph, nullptr, nullptr, 0));
      st.gkey = key;
    }
    for (int i = 0; i < p->steps; ++i) HIPK(hipGraphLaunch(st.gexec, hs));
  } else {
    for (int i = 0; i < p->steps; ++i) guided_step(s, st, g, p->steps, p->opt);
  }
}

// final decode (marigold_dc.py:969-985) of the latents in x8[..., 4:8] with the learned affine in st.affine
void final_decode(dc_session* s, PlanState& st, const Geo& g, float* dense) {
  Exec& ex = s->ex;
  DecoderPlan& dp = *st.dec;
  dp.set_rows(nullptr);
  const long P = (long)g.n * g.h * g.w;
  DCK(dc_taesd_clamp_fwd(st.unet->x8.col(4).p, 8, P, dp.tin.p, ex.stream));
  dp.forward();
  DCK(dc_final_dense(dp.out.p, 8, g.n, g.PH, g.PW, g.RH, g.RW, g.H, g.W, st.params, st.affine, 0, dense, ex.stream));
}

void encode_into(dc_session* s, PlanState& st, const Geo& g, const void* imgs_u8) {
  Exec& ex = s->ex;
  DevMem scratch;
  RB img8(scratch.alloc((size_t)g.n * g.PH * g.PW * 8 * 2, false), 8);
  DCK(dc_preprocess_image(imgs_u8, g.n, g.H, g.W, g.RH, g.RW, g.PH, g.PW, 1, img8.p, ex.stream));
  taesd_encode(s->taesd, ex, scratch, img8, g.n, g.PH, g.PW, st.unet->x8.col(0));
  HIPK(hipStreamSynchronize(ex.stream));  // scratch is freed on return
}

template <typename F>
int guarded(dc_session* s, void* user_stream, F&& f) {
  if (!s) return kErrArg;
  try {
    HIPK(hipSetDevice(s->device));
    if (!s->loaded) throw DcError(kErrArg, "no weights loaded (dc_load_weights)");
    // order the session stream after the caller's work, and the caller's stream after ours.  On success the join's
    // statuses are checked (join() throws on a failed record / wait); when f() or the join throws after queueing
    // work that reads the caller's buffers, the destructor still joins the streams, best effort, and destroys the
    // event on every exit path
    struct StreamJoin {
      hipEvent_t e = nullptr;
      hipStream_t sess, user;
      void join() {
        HIPK(hipEventRecord(e, sess));
        HIPK(hipStreamWaitEvent(user, e, 0));
        const hipError_t d = hipEventDestroy(e);
        e = nullptr;
        if (d != hipSuccess) throw DcError(kErrLaunch, std::string("hipEventDestroy: ") + hipGetErrorString(d));
      }
      ~StreamJoin() {
        if (!e) return;
        (void)hipEventRecord(e, sess);
        (void)hipStreamWaitEvent(user, e, 0);
        (void)hipEventDestroy(e);
      }
    } join{nullptr, s->stream, (hipStream_t)user_stream};
    HIPK(hipEventCreateWithFlags(&join.e, hipEventDisableTiming));
    HIPK(hipEventRecord(join.e, (hipStream_t)user_stream));
    HIPK(hipStreamWaitEvent(s->stream, join.e, 0));
    f();
    join.join();
    s->err.clear();
    return kOK;
  } catch (const DcError& e) {
    s->err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    s->err = e.what();
    return kErrArg;
  }
}

}  // namespace

// ------------------------------------------------------------------ C ABI
extern "C" void dc_sample_params_default(dc_sample_params* p) {
  if (!p) return;
  p->max_depth = 120.0f;
  p->min_depth = 0.0f;
  p->norm = 0;
  p->projection = 0;
  p->inv = 0;
  p->interp = 0;
  p->steps = 50;
  p->resolution = 768;
  p->opt = 0;
  p->lr_latent = 0.05;
  p->lr_scaling = 0.005;
  p->beta = 0.9f;
  p->use_graph = 1;
}

extern "C" int dc_latent_hw(int H, int W, int resolution, int* h, int* w) {
  if (H <= 0 || W <= 0 || resolution <= 0 || !h || !w) return kErrArg;
  const Geo g = geometry(1, H, W, resolution);
  *h = g.h;
  *w = g.w;
  return kOK;
}

extern "C" int dc_create(dc_session** out, int device) {
  if (!out) return kErrArg;
  *out = nullptr;
  try {
    HIPK(hipSetDevice(device));
    auto s = std::make_unique<dc_session>();
    s->device = device;
    HIPK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    s->ex.stream = s->stream;
    s->ex.ws_bytes = 96LL << 20;   // ops.Ctx: 96 MB fp32 scratch, zero-filled (split-K counters in its last 64 KB)
    s->ex.ws = (float*)s->cmem.alloc((size_t)s->ex.ws_bytes);
    s->ex.step = (int*)s->cmem.alloc(4);
    const char* sd = getenv("DC_SPARSE_DECODE");
    s->sparse_decode = !(sd && std::string(sd) == "0");
    *out = s.release();
    return kOK;
  } catch (const DcError& e) {
    return e.code;
  }
}

extern "C" int dc_destroy(dc_session* s) {
  if (!s) return kErrArg;
  (void)hipSetDevice(s->device);
  (void)hipStreamSynchronize(s->stream);
  s->plans.clear();
  hipStream_t st = s->stream;
  delete s;
  if (st) (void)hipStreamDestroy(st);
  return kOK;
}

extern "C" const char* dc_session_error(const dc_session* s) { return s ? s->err.c_str() : "null session"; }

extern "C" int dc_load_weights(dc_session* s, const char* dir, const char* tuned_table) {
  if (!s || !dir) return kErrArg;
  try {
    HIPK(hipSetDevice(s->device));
    const std::string d(dir);
    // UNet config (diffusers config.json; Marigold v1-0 defaults)
    UNetCfg cfg;
    const std::string cj = read_file(d + "/unet/config.json");
    if (!cj.empty()) {
      dcjson::Value c = dcjson::parse(cj);
      if (auto v = c.get("block_out_channels")) { cfg.ch.clear(); for (auto& x : v->arr) cfg.ch.push_back((int)x.as_int()); }
      if (auto v = c.get("attention_head_dim")) {
        cfg.heads.clear();
        if (v->kind == dcjson::Value::Arr) for (auto& x : v->arr) cfg.heads.push_back((int)x.as_int());
        else cfg.heads.assign(cfg.ch.size(), (int)v->as_int());
      }
      if (auto v = c.get("cross_attention_dim")) cfg.cross = (int)v->as_int();
      if (auto v = c.get("layers_per_block")) cfg.layers = (int)v->as_int();
      if (auto v = c.get("norm_num_groups")) if (v->as_int() != 32) throw DcError(kErrArg, "norm_num_groups must be 32");
      if (auto v = c.get("down_block_types")) {
        cfg.down_attn.clear();
        for (auto& x : v->arr) cfg.down_attn.push_back(x.str.find("CrossAttn") != std::string::npos);
      }
      if (auto v = c.get("up_block_types")) {
        cfg.up_attn.clear();
        for (auto& x : v->arr) cfg.up_attn.push_back(x.str.find("CrossAttn") != std::string::npos);
      }
    }
    if (cfg.heads.size() != cfg.ch.size() || cfg.down_attn.size() != cfg.ch.size() || cfg.up_attn.size() != cfg.ch.size())
      throw DcError(kErrArg, "inconsistent UNet config");
    SafeTensors emb_st(d + "/empty_text_embedding.safetensors");
    HostTensor emb = emb_st.get("embedding");
    const int cross = (int)emb.shape.back();
    const int ntok = (int)(emb.numel() / cross);
    if (cross != cfg.cross) throw DcError(kErrArg, "text embedding width != cross_attention_dim");
    // a failed (re)load leaves the session unloaded (never half-loaded): the new weights go into locals and
    // are swapped in only once everything has loaded
    s->loaded = false;
    s->plans.clear();
    s->unet = UNetW();
    s->taesd = TAESDW();
    s->wmem = DevMem();
    DevMem wmem;
    UNetW unet;
    unet.cfg = cfg;
    TAESDW taesd;
    {
      SafeTensors ust(d + "/unet/diffusion_pytorch_model.safetensors");
      Loader L(ust, wmem);
      load_unet(unet, L, emb.data, ntok);
    }
    {
      std::string tp = d + "/taesd/diffusion_pytorch_model.safetensors";
      if (read_file(tp).empty()) tp = d + "/vae/diffusion_pytorch_model.safetensors";
      SafeTensors tst(tp);
      Loader L(tst, wmem);
      load_taesd(taesd, L);
    }
    s->wmem = std::move(wmem);
    s->unet = std::move(unet);
    s->taesd = std::move(taesd);
    s->ex.tuned.clear();
    s->ex.table_keys.clear();
    s->ex.table_choices.clear();
    s->ex.picked.clear();
    const char* nn = getenv("DC_GEMM_NN");
    s->ex.nn = !(nn && std::string(nn) == "0");
    if (tuned_table && *tuned_table) load_tuned(s->ex, tuned_table);
    s->loaded = true;
    s->err.clear();
    return kOK;
  } catch (const DcError& e) {
    s->err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    s->err = e.what();
    return kErrArg;
  }
}

extern "C" int dc_encode(dc_session* s, const void* imgs_u8, int n, int H, int W, int resolution, void* latents,
                         void* stream) {
  return guarded(s, stream, [&]() {
    if (!imgs_u8 || !latents || n <= 0 || H <= 0 || W <= 0 || resolution <= 0) throw DcError(kErrArg, "bad arguments");
    const Geo g = geometry(n, H, W, resolution);
    PlanState& st = plan(s, n, g.h, g.w);
    encode_into(s, st, g, imgs_u8);
    DCK(dc_nhwc_to_nchw(st.unet->x8.p, 8, n, (long long)g.h * g.w, 4, latents, s->stream));
  });
}

extern "C" int dc_guided_sample(dc_session* s, const void* img_latents, const void* noise, int noise_n,
                                const void* prev, const float* sparses, int n, int H, int W,
                                const dc_sample_params* p, void* latents_out, float* affine_out, void* stream) {
  return guarded(s, stream, [&]() {
    check_params(p);
    if (!img_latents || !noise || !sparses || !latents_out || n <= 0 || H <= 0 || W <= 0)
      throw DcError(kErrArg, "bad arguments");
    if (noise_n != 1 && noise_n != n) throw DcError(kErrArg, "noise must hold 1 or n draws");
    const Geo g = geometry(n, H, W, p->resolution);
    PlanState& st = plan(s, n, g.h, g.w);
    DCK(dc_nchw_to_nhwc(img_latents, n, (long long)g.h * g.w, 4, st.unet->x8.p, 8, s->stream));
    sample(s, st, g, noise, noise_n, prev, sparses, p);
    DCK(dc_nhwc_to_nchw(st.unet->x8.col(4).p, 8, n, (long long)g.h * g.w, 4, latents_out, s->stream));
    if (affine_out) HIPK(hipMemcpyAsync(affine_out, st.affine, (size_t)n * 2 * 4, hipMemcpyDeviceToDevice, s->stream));
  });
}

extern "C" int dc_decode_dense(dc_session* s, const void* latents, const float* affine, const float* sparses, int n,
                               int H, int W, const dc_sample_params* p, float* dense_out, void* stream) {
  return guarded(s, stream, [&]() {
    check_params(p);
    if (!latents || !affine || !sparses || !dense_out || n <= 0 || H <= 0 || W <= 0)
      throw DcError(kErrArg, "bad arguments");
    const Geo g = geometry(n, H, W, p->resolution);
    PlanState& st = plan(s, n, g.h, g.w);
    if (st.tab_hw != (long)H * W) {
      st.tabs = DevMem();
      st.idx = (int*)st.tabs.alloc((size_t)n * H * W * 4, false);
      st.gval = (float*)st.tabs.alloc((size_t)n * H * W * 4, false);
      st.cnt = (int*)st.tabs.alloc(n * 4, false);
      st.params = (float*)st.tabs.alloc(n * 8 * 4, false);
      st.coef = st.adam = nullptr;
      st.tab_hw = H * W;
      st.tab_steps = 0;
      if (st.gexec) { (void)hipGraphExecDestroy(st.gexec); st.gexec = nullptr; }
      if (st.graph) { (void)hipGraphDestroy(st.graph); st.graph = nullptr; }
    }
    // the de-normalisation needs the sparse statistics of dc_sparse_setup (marigold_dc.py:706-756, 981-985)
    DCK(dc_sparse_setup(sparses, n, H, W, p->norm, p->min_depth, p->max_depth, nullptr, p->projection, p->inv,
                        p->interp, st.idx, st.gval, st.cnt, st.params, s->stream));
    DCK(dc_nchw_to_nhwc(latents, n, (long long)g.h * g.w, 4, st.unet->x8.col(4).p, 8, s->stream));
    HIPK(hipMemcpyAsync(st.affine, affine, (size_t)n * 2 * 4, hipMemcpyDeviceToDevice, s->stream));
    final_decode(s, st, g, dense_out);
  });
}

extern "C" int dc_complete(dc_session* s, const void* imgs_u8, const float* sparses, int n, int H, int W,
                           const void* noise, int noise_n, const void* prev, const dc_sample_params* p,
                           float* dense_out, void* latents_out, void* stream) {
  return guarded(s, stream, [&]() {
    check_params(p);
    if (!imgs_u8 || !sparses || !noise || !dense_out || n <= 0 || H <= 0 || W <= 0)
      throw DcError(kErrArg, "bad arguments");
    if (noise_n != 1 && noise_n != n) throw DcError(kErrArg, "noise must hold 1 or n draws");
    const Geo g = geometry(n, H, W, p->resolution);
    PlanState& st = plan(s, n, g.h, g.w);
    // pipeline.__call__ order: latent init (inside sample), preprocess + TAESD encoder into x8[..., 0:4], sparse
    // setup, row sets, tables, loop, final decode
    encode_into(s, st, g, imgs_u8);
    sample(s, st, g, noise, noise_n, prev, sparses, p);
    final_decode(s, st, g, dense_out);
    if (latents_out)
      DCK(dc_nhwc_to_nchw(st.unet->x8.col(4).p, 8, n, (long long)g.h * g.w, 4, latents_out, s->stream));
  });
}
