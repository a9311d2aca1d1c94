// Host-side robustness driver, built under ASan + UBSan by tests/test_sanitizers.py (CPU; SURVEY.md §5
// "race detection / sanitizers": host ASan/UBSan on the C-ABI shim).
//
// Exercises the host code of libdcamd that parses untrusted input or computes tables without a GPU:
//   * dcjson::parse (config.json, safetensors headers, the tuned GEMM table) on crafted and mutated input;
//   * dcst::SafeTensors (the native session's weight reader) on a valid file and on crafted / mutated headers;
//   * dc_schedule_tables / dc_timestep_embedding / dc_fold_cross_attention on valid and invalid arguments.
// Every input must either parse or throw std::exception (and every bad argument return non-zero): a crash, an
// out-of-bounds access, a leak or undefined behaviour fails the run.  Exit status 0 = clean.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dcamd.h"
#include "json_mini.h"
#include "safetensors_mini.h"

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                 \
  do {                                   \
    if (!(cond)) {                       \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");             \
      ++g_fail;                          \
    }                                    \
  } while (0)

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 6364136223846793005ull + 1442695040888963407ull) {}
  uint32_t next() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
  }
  uint32_t below(uint32_t n) { return n ? next() % n : 0; }
};

std::string mutate(const std::string& in, Rng& r) {
  std::string s = in;
  const int edits = 1 + (int)r.below(4);
  static const char alphabet[] = "{}[]\",:\\u0123456789eE+-.tfnrl \n";
  for (int e = 0; e < edits; ++e) {
    const uint32_t kind = r.below(4);
    const size_t pos = s.empty() ? 0 : r.below((uint32_t)s.size());
    if (kind == 0 && !s.empty()) s[pos] = alphabet[r.below(sizeof(alphabet) - 1)];
    else if (kind == 1) s.insert(pos, 1, alphabet[r.below(sizeof(alphabet) - 1)]);
    else if (kind == 2 && !s.empty()) s.erase(pos, 1 + r.below(8));
    else s = s.substr(0, pos);
  }
  return s;
}

void touch(const dcjson::Value& v, int depth = 0) {
  if (depth > 200) return;
  try {
    (void)v.as_int();
  } catch (const std::exception&) {
  }
  for (auto& a : v.arr) touch(a, depth + 1);
  for (auto& kv : v.obj) touch(kv.second, depth + 1);
  (void)v.get("shape");
}

int json_parses = 0, json_rejects = 0;
void json_case(const std::string& s) {
  try {
    const dcjson::Value v = dcjson::parse(s);
    touch(v);
    ++json_parses;
  } catch (const std::exception&) {
    ++json_rejects;
  }
}

void fuzz_json() {
  const std::vector<std::string> seeds = {
      R"({"in_channels": 8, "block_out_channels": [320, 640, 1280, 1280], "attention_head_dim": [5, 10, 20, 20],)"
      R"( "cross_attention_dim": 1024, "use_linear_projection": true, "name": "unet\u00e9\n"})",
      R"({"w": {"dtype": "BF16", "shape": [2, 3], "data_offsets": [0, 12]}, "__metadata__": {"format": "pt"}})",
      R"([{"mode": 0, "m": 6912, "algo": 3, "splitk": -2}, {"mode": 1, "m": 432, "algo": 13, "splitk": 4}])",
      R"({"a": [1.5e3, -2, true, false, null, "x\"y\\z"], "b": {}})"};
  const std::vector<std::string> crafted = {
      "", "{", "[", "}", "\"", "\"\\", "\"\\u12", "{\"a\"", "{\"a\":", "{\"a\":}", "[1,]", "[,1]", "{,}", "nul",
      "tru", "1e999", "-1e999", "1e30", "-4.7e18", "4.5e18", "NaN", "[1 2]", "{\"a\" 1}", "\"abc", "0x10",
      std::string(5000, '['), std::string(5000, '{'), std::string(3, '\0'), "[\"\\u\"]", "  \n\t "};
  for (auto& c : crafted) json_case(c);
  for (auto& s : seeds) json_case(s);
  Rng r(2024);
  for (int it = 0; it < 20000; ++it) json_case(mutate(seeds[it % seeds.size()], r));
  CHECK(json_parses >= 4, "valid JSON seeds must parse (%d parsed)", json_parses);
  // the out-of-range integer guard
  bool threw = false;
  try {
    (void)dcjson::parse("1e30").as_int();
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw, "as_int(1e30) must throw");
  printf("json: %d parsed, %d rejected\n", json_parses, json_rejects);
}

// ---------------------------------------------------------------- safetensors
std::string st_file(const std::string& header, const std::string& data) {
  std::string f(8, '\0');
  const uint64_t hl = header.size();
  memcpy(&f[0], &hl, 8);
  return f + header + data;
}

void write_file(const std::string& path, const std::string& bytes) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    ++g_fail;
    return;
  }
  fwrite(bytes.data(), 1, bytes.size(), f);
  fclose(f);
}

int st_ok = 0, st_rejects = 0;
void st_case(const std::string& path, const std::string& bytes) {
  write_file(path, bytes);
  try {
    dcst::SafeTensors st(path);
    for (const char* k : {"a", "b", "c", "d", "__metadata__", "missing"}) {
      try {
        const dcst::HostTensor t = st.get(k);
        float acc = 0.0f;
        for (float v : t.data) acc += v;
        (void)acc;
        ++st_ok;
      } catch (const std::exception&) {
        ++st_rejects;
      }
    }
  } catch (const std::exception&) {
    ++st_rejects;
  }
}

void fuzz_safetensors(const std::string& dir) {
  const std::string path = dir + "/fuzz.safetensors";
  // valid: a F32[2,2], b BF16[3], c F16[2], d F64[1]
  std::string data;
  const float a[4] = {1.0f, -2.0f, 3.5f, 0.25f};
  data.append((const char*)a, 16);
  const uint16_t b[3] = {0x3f80, 0xc000, 0x4040};  // 1, -2, 3
  data.append((const char*)b, 6);
  const uint16_t c[2] = {0x3c00, 0xbc00};  // 1, -1
  data.append((const char*)c, 4);
  const double d[1] = {6.5};
  data.append((const char*)d, 8);
  const std::string header =
      R"({"a": {"dtype": "F32", "shape": [2, 2], "data_offsets": [0, 16]},)"
      R"( "b": {"dtype": "BF16", "shape": [3], "data_offsets": [16, 22]},)"
      R"( "c": {"dtype": "F16", "shape": [2], "data_offsets": [22, 26]},)"
      R"( "d": {"dtype": "F64", "shape": [1], "data_offsets": [26, 34]}, "__metadata__": {"format": "pt"}})";
  const std::string good = st_file(header, data);
  write_file(path, good);
  try {
    dcst::SafeTensors st(path);
    const auto ta = st.get("a"), tb = st.get("b"), tc = st.get("c"), td = st.get("d");
    CHECK(ta.numel() == 4 && ta.data[2] == 3.5f, "F32 tensor");
    CHECK(tb.data[1] == -2.0f && tb.data[2] == 3.0f, "BF16 tensor");
    CHECK(tc.data[0] == 1.0f && tc.data[1] == -1.0f, "F16 tensor");
    CHECK(td.data[0] == 6.5f, "F64 tensor");
    CHECK(st.has("a") && !st.has("__metadata__") && !st.has("zz"), "has()");
  } catch (const std::exception& e) {
    CHECK(false, "valid file rejected: %s", e.what());
  }
  // crafted corruptions: each must be rejected (no crash)
  auto entry = [&](const std::string& e) { return st_file("{\"a\": " + e + "}", data); };
  const std::vector<std::string> bad = {
      std::string(4, '\0'),                                                        // shorter than the length
      st_file(header, data).substr(0, 8 + header.size() - 1),                      // header cut
      [&] { std::string f = good; const uint64_t hl = ~0ull; memcpy(&f[0], &hl, 8); return f; }(),
      [&] { std::string f = good; const uint64_t hl = 1ull << 40; memcpy(&f[0], &hl, 8); return f; }(),
      st_file("[1, 2]", data),                                                     // header not an object
      entry(R"({"dtype": "F32", "shape": [2, 2], "data_offsets": [0, 1600]})"),    // past the end
      entry(R"({"dtype": "F32", "shape": [2, 2], "data_offsets": [16, 0]})"),      // reversed
      entry(R"({"dtype": "F32", "shape": [2, 2], "data_offsets": [-16, 0]})"),     // negative
      entry(R"({"dtype": "F32", "shape": [2, 3], "data_offsets": [0, 16]})"),      // numel mismatch
      entry(R"({"dtype": "F32", "shape": [-1, -4], "data_offsets": [0, 16]})"),    // negative dims
      entry(R"({"dtype": "F32", "shape": [4294967296, 4294967296], "data_offsets": [0, 16]})"),  // overflow
      entry(R"({"dtype": "I64", "shape": [2], "data_offsets": [0, 16]})"),         // unsupported dtype
      entry(R"({"dtype": 7, "shape": [4], "data_offsets": [0, 16]})"),
      entry(R"({"dtype": "F32", "shape": 4, "data_offsets": [0, 16]})"),
      entry(R"({"dtype": "F32", "shape": [4], "data_offsets": [0]})"),
      entry(R"([1, 2, 3])"),
      entry(R"({"dtype": "F32", "shape": [4], "data_offsets": [0, 1e300]})"),
  };
  for (size_t i = 0; i < bad.size(); ++i) {
    write_file(path, bad[i]);
    bool rejected = false;
    try {
      dcst::SafeTensors st(path);
      (void)st.get("a");
    } catch (const std::exception&) {
      rejected = true;
    }
    CHECK(rejected, "corrupt safetensors case %zu accepted", i);
  }
  // mutated headers (length kept consistent and not), mutated data lengths
  Rng r(7);
  for (int it = 0; it < 3000; ++it) {
    const std::string h = mutate(header, r);
    std::string dd = data;
    if (it % 3 == 0) dd = dd.substr(0, r.below((uint32_t)dd.size() + 1));
    std::string f = st_file(h, dd);
    if (it % 7 == 0 && f.size() >= 8) {
      const uint64_t hl = r.next() % (f.size() + 16);
      memcpy(&f[0], &hl, 8);
    }
    st_case(path, f);
  }
  printf("safetensors: %d tensors read, %d rejected\n", st_ok, st_rejects);
}

// ---------------------------------------------------------------- host tables
void host_tables() {
  std::vector<long long> ts(1001);
  std::vector<float> coef(4 * 1001), adam(4 * 1001);
  for (int steps : {-5, 0, 1, 2, 3, 7, 10, 49, 50, 333, 999, 1000, 1001, 5000})
    for (int opt = -1; opt <= 3; ++opt) {
      const int rc = dc_schedule_tables(steps, 0.05, 0.005, opt, ts.data(), coef.data(), adam.data());
      const bool valid = steps >= 1 && steps <= 1000 && opt >= 0 && opt <= 2;
      CHECK((rc == 0) == valid, "dc_schedule_tables(%d, opt %d) rc %d", steps, opt, rc);
      if (valid) {
        for (int s = 0; s < steps; ++s) {
          CHECK(ts[s] >= 0 && ts[s] < 1000, "timestep range");
          CHECK(std::isfinite(coef[4 * s]) && coef[4 * s] > 0.0f && std::isfinite(adam[4 * s]), "finite tables");
        }
      }
    }
  CHECK(dc_schedule_tables(10, 0.05, 0.005, 0, nullptr, coef.data(), adam.data()) != 0, "null timesteps");
  CHECK(dc_schedule_tables(10, 0.05, 0.005, 0, ts.data(), nullptr, adam.data()) != 0, "null coef");

  std::vector<float> emb(4 * 1280);
  const long long t4[4] = {999, 0, 19, 500};
  for (int dim : {-2, 0, 1, 2, 3, 320, 1280}) {
    const int rc = dc_timestep_embedding(t4, 4, dim, emb.data());
    CHECK((rc == 0) == (dim >= 2 && dim % 2 == 0), "dc_timestep_embedding dim %d rc %d", dim, rc);
  }
  CHECK(dc_timestep_embedding(nullptr, 4, 320, emb.data()) != 0, "null timesteps (embedding)");
  CHECK(dc_timestep_embedding(t4, 0, 320, emb.data()) != 0, "n = 0");

  Rng r(11);
  int folds = 0;
  for (int it = 0; it < 200; ++it) {
    const int heads = 1 + (int)r.below(4), hd = 1 + (int)r.below(8);
    const int inner = heads * hd, c = 1 + (int)r.below(24), cross = 1 + (int)r.below(16), cout = 1 + (int)r.below(24);
    std::vector<float> wq((size_t)inner * c), wk((size_t)inner * cross), wv((size_t)inner * cross),
        wo((size_t)cout * inner), bo(cout), ctx(2 * (size_t)cross), U((size_t)heads * c), D((size_t)heads * cout),
        c0(cout);
    for (auto* v : {&wq, &wk, &wv, &wo, &bo, &ctx})
      for (float& x : *v) x = (float)((int)r.below(2001) - 1000) / 1000.0f;
    const int rc = dc_fold_cross_attention(wq.data(), wk.data(), wv.data(), wo.data(), bo.data(), ctx.data(), 2, inner,
                                           c, cross, cout, heads, U.data(), D.data(), c0.data());
    CHECK(rc == 0, "fold rc %d", rc);
    for (float x : U) CHECK(std::isfinite(x), "U finite");
    ++folds;
  }
  float z[4] = {};
  CHECK(dc_fold_cross_attention(z, z, z, z, z, z, 3, 2, 2, 2, 2, 1, z, z, z) != 0, "ntok != 2");
  CHECK(dc_fold_cross_attention(z, z, z, z, z, z, 2, 3, 2, 2, 2, 2, z, z, z) != 0, "inner %% heads");
  CHECK(dc_fold_cross_attention(z, z, z, z, z, z, 2, 2, 0, 2, 2, 1, z, z, z) != 0, "c = 0");
  CHECK(dc_fold_cross_attention(z, z, z, z, z, z, 2, 2, 2, 2, 2, 1, nullptr, z, z) != 0, "null U");
  printf("host tables: %d folds\n", folds);
}

}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  fuzz_json();
  fuzz_safetensors(dir);
  host_tables();
  printf("%s (%d failures)\n", g_fail ? "FAILED" : "clean", g_fail);
  return g_fail ? 1 : 0;
}
