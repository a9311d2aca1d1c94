// Read-only safetensors reader (mmap) for the native session's weight loading (session.cpp).  Host-only C++
// with no HIP dependency, so the CPU sanitizer test (tests/test_sanitizers.py) builds it under
// ASan/UBSan and feeds it malformed files.  Every header field is validated before a byte of tensor data is
// touched: header length inside the file, dtype known, non-negative shape with an overflow-free element count,
// data_offsets ordered, inside the data section and exactly numel * itemsize long.  Violations throw
// std::runtime_error (the session maps that to DC_ERR_ARG + dc_session_error()).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "json_mini.h"

namespace dcst {

inline float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

inline float half2f(uint16_t h) {
  const uint32_t s = (h >> 15) & 1u, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 0x400u), (int)e - 25);
  return s ? -v : v;
}

struct HostTensor {
  std::vector<long> shape;
  std::vector<float> data;  // converted to fp32
  long numel() const {
    long n = 1;
    for (long s : shape) n *= s;
    return n;
  }
};

class SafeTensors {
 public:
  explicit SafeTensors(const std::string& path) : path_(path) {
    fd_ = open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0 || st.st_size < 8) fail("file shorter than the 8-byte header length");
    size_ = (size_t)st.st_size;
    void* m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (m == MAP_FAILED) fail("cannot map");
    base_ = (const char*)m;
    uint64_t hl;
    memcpy(&hl, base_, 8);
    if (hl > size_ - 8) fail("header length beyond the end of the file");
    try {
      head_ = dcjson::parse(std::string(base_ + 8, (size_t)hl));
    } catch (const std::exception& e) {
      fail(std::string("header: ") + e.what());
    }
    if (head_.kind != dcjson::Value::Obj) fail("header is not a JSON object");
    data_ = base_ + 8 + hl;
    data_bytes_ = size_ - 8 - (size_t)hl;
  }
  SafeTensors(const SafeTensors&) = delete;
  SafeTensors& operator=(const SafeTensors&) = delete;
  ~SafeTensors() { release(); }

  bool has(const std::string& k) const { return k != "__metadata__" && head_.get(k) != nullptr; }

  HostTensor get(const std::string& k) const {
    const dcjson::Value* v = k == "__metadata__" ? nullptr : head_.get(k);
    if (!v) throw std::runtime_error("missing tensor '" + k + "' in " + path_);
    if (v->kind != dcjson::Value::Obj) bad(k, "entry is not an object");
    const dcjson::Value& shp = v->at("shape");
    const dcjson::Value& dtv = v->at("dtype");
    const dcjson::Value& offv = v->at("data_offsets");
    if (shp.kind != dcjson::Value::Arr || dtv.kind != dcjson::Value::Str || offv.kind != dcjson::Value::Arr ||
        offv.arr.size() != 2)
      bad(k, "malformed shape / dtype / data_offsets");
    HostTensor t;
    long n = 1;
    for (auto& s : shp.arr) {
      const long long d = s.as_int();
      if (d < 0 || (d > 0 && n > (1LL << 40) / d)) bad(k, "bad shape");
      n *= (long)d;
      t.shape.push_back((long)d);
    }
    const std::string& dt = dtv.str;
    const int item = dt == "F32" ? 4 : dt == "BF16" ? 2 : dt == "F16" ? 2 : dt == "F64" ? 8 : 0;
    if (!item) bad(k, "unsupported dtype " + dt);
    const long long o0 = offv.arr[0].as_int(), o1 = offv.arr[1].as_int();
    if (o0 < 0 || o1 < o0 || (unsigned long long)o1 > data_bytes_) bad(k, "data_offsets outside the data section");
    if (o1 - o0 != (long long)n * item) bad(k, "data_offsets length != numel * itemsize");
    const char* p = data_ + o0;
    t.data.resize((size_t)n);
    if (item == 4) {
      memcpy(t.data.data(), p, (size_t)n * 4);
    } else if (dt == "BF16") {
      for (long i = 0; i < n; ++i) { uint16_t h; memcpy(&h, p + 2 * i, 2); t.data[i] = bf2f(h); }
    } else if (dt == "F16") {
      for (long i = 0; i < n; ++i) { uint16_t h; memcpy(&h, p + 2 * i, 2); t.data[i] = half2f(h); }
    } else {
      for (long i = 0; i < n; ++i) { double d; memcpy(&d, p + 8 * i, 8); t.data[i] = (float)d; }
    }
    return t;
  }

 private:
  std::string path_;
  int fd_ = -1;
  size_t size_ = 0, data_bytes_ = 0;
  const char* base_ = nullptr;
  const char* data_ = nullptr;
  dcjson::Value head_;

  void release() {
    if (base_) munmap((void*)base_, size_);
    if (fd_ >= 0) close(fd_);
    base_ = nullptr;
    fd_ = -1;
  }
  [[noreturn]] void fail(const std::string& what) {
    release();
    throw std::runtime_error("bad safetensors file " + path_ + ": " + what);
  }
  [[noreturn]] void bad(const std::string& k, const std::string& what) const {
    throw std::runtime_error("bad safetensors entry '" + k + "' in " + path_ + ": " + what);
  }
};

}  // namespace dcst
