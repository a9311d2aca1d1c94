// Pixel row sets of the sparse-aware TAESD decode (gfx950).
//
// With the point losses (l1 / l2, marigold_dc.py:195-205) the guided step reads the decoded map only at
// the resize taps of the sparse pixels (dc_sparse_loss / dc_sparse_loss_cf), so the decoder's
// full-resolution layers need their outputs only inside the taps' receptive fields: S0 = the tap
// pixels, S(k+1) = S(k) dilated by the 3x3 kernel.  These kernels build the sets as sorted row lists
// for dc_conv_gemm's `rows` field:
//   tap_mask_kernel      S0 as a byte mask [nb][ph][pw] (the taps of sample_affine in guidance.hip)
//   dilate_kernel        3x3 dilation within each frame
//   chunk_count / scan / compact   mask -> sorted row indices (1024-pixel chunks, exclusive scans)
#include "common.h"
#include "../../include/dcamd.h"

namespace {

constexpr int kChunk = 1024;

// upsample_bilinear2d (align_corners=False) / nearest source taps, as guidance.hip's sample_affine
__device__ void mark_taps(unsigned char* m, int PH, int PW, int RH, int RW, int H, int W, int y, int x, int nearest) {
  auto nsrc = [](int dst, int in, int out) {
    if (in == out) return dst;
    if (out == 2 * in) return dst >> 1;
    const float scale = (float)in / (float)out;
    const int s = (int)floorf((float)dst * scale);
    return s < in - 1 ? s : in - 1;
  };
  if (nearest) {
    m[(long)nsrc(y, RH, H) * PW + nsrc(x, RW, W)] = 1;
    return;
  }
  if (RH == H && RW == W) {
    m[(long)y * PW + x] = 1;
    return;
  }
  const float rh = (float)RH / H, rw = (float)RW / W;
  float sy = rh * (y + 0.5f) - 0.5f;
  sy = sy < 0.0f ? 0.0f : sy;
  float sx = rw * (x + 0.5f) - 0.5f;
  sx = sx < 0.0f ? 0.0f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + ((y0 < RH - 1) ? 1 : 0), x1 = x0 + ((x0 < RW - 1) ? 1 : 0);
  m[(long)y0 * PW + x0] = 1;
  m[(long)y0 * PW + x1] = 1;
  m[(long)y1 * PW + x0] = 1;
  m[(long)y1 * PW + x1] = 1;
}

__global__ void tap_mask_kernel(const int* idx, const int* cnt, const float* params, int PH, int PW, int RH, int RW,
                                int H, int W, unsigned char* mask) {
  const int n = blockIdx.y;
  const long HW = (long)H * W;
  const int nearest = ((int)params[n * 8 + 7] >> 3) & 1;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < cnt[n]; k += gridDim.x * blockDim.x) {
    const int p = idx[n * HW + k];
    mark_taps(mask + (long)n * PH * PW, PH, PW, RH, RW, H, W, p / W, p - (p / W) * W, nearest);
  }
}

__global__ void dilate_kernel(const unsigned char* in, int PH, int PW, long total, unsigned char* out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long hw = (long)PH * PW;
    const long n = i / hw;
    const int r = (int)(i - n * hw), y = r / PW, x = r - (r / PW) * PW;
    const unsigned char* f = in + n * hw;
    unsigned char v = 0;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xx = x + dx;
        if (yy >= 0 && yy < PH && xx >= 0 && xx < PW) v |= f[(long)yy * PW + xx];
      }
    out[i] = v;
  }
}

// exclusive prefix of `flag` over the block (1024 threads), block total in *tot
__device__ int block_excl_scan(int flag, int* sh, int* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(flag);
  const int before = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) sh[w] = __popcll(bal);
  __syncthreads();
  int off = 0, all = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    off += k < w ? sh[k] : 0;
    all += sh[k];
  }
  *tot = all;
  return off + before;
}

__global__ void chunk_count_kernel(const unsigned char* mask, long total, int* ccnt) {
  __shared__ int sh[16];
  const long i = (long)blockIdx.x * kChunk + threadIdx.x;
  int tot;
  block_excl_scan(i < total && mask[i], sh, &tot);
  if (threadIdx.x == 0) ccnt[blockIdx.x] = tot;
}

// one block: exclusive scan of the chunk counts (in place -> offsets), count[0] = total
__global__ void chunk_scan_kernel(int* ccnt, int nchunk, int* count) {
  __shared__ int sh[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nchunk; base += kChunk) {
    const int i = base + threadIdx.x;
    const int v = i < nchunk ? ccnt[i] : 0;
    // block scan of values (not flags): per-wave inclusive scan by shuffles, then wave offsets
    int x = v;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(x, o, 64);
      if (lane >= o) x += t;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int off = carry;
    for (int k = 0; k < w; ++k) off += sh[k];
    int all = 0;
    for (int k = 0; k < 16; ++k) all += sh[k];
    if (i < nchunk) ccnt[i] = off + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) count[0] = carry;
}

__global__ void compact_kernel(const unsigned char* mask, long total, const int* coff, int* rows) {
  __shared__ int sh[16];
  const long i = (long)blockIdx.x * kChunk + threadIdx.x;
  const int flag = i < total && mask[i];
  int tot;
  const int pos = block_excl_scan(flag, sh, &tot);
  if (flag) rows[coff[blockIdx.x] + pos] = (int)i;
}

// rows[count .. pad_to) = rows[count - 1]: padded launches recompute the last pixel (identical writes)
__global__ void pad_rows_kernel(int* rows, const int* count, int pad_to) {
  const int c = count[0];
  for (int i = c + blockIdx.x * blockDim.x + threadIdx.x; i < pad_to; i += gridDim.x * blockDim.x)
    rows[i] = c > 0 ? rows[c - 1] : 0;
}

}  // namespace

extern "C" int dc_tap_mask(const int* idx, const int* cnt, const float* params, int nb, int ph, int pw, int rh,
                           int rw, int h, int w, unsigned char* mask, void* stream) {
  if (!idx || !cnt || !params || !mask || nb <= 0 || rh > ph || rw > pw || h <= 0 || w <= 0) return DC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (dc_memset_async(mask, 0, (long long)nb * ph * pw, stream) != DC_OK) return DC_ERR_LAUNCH;
  const long HW = (long)h * w;
  const dim3 g((unsigned)min((HW + 255) / 256, 1024L), nb);
  hipLaunchKernelGGL(tap_mask_kernel, g, dim3(256), 0, st, idx, cnt, params, ph, pw, rh, rw, h, w, mask);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_dilate_mask(const unsigned char* in, int nb, int ph, int pw, unsigned char* out, void* stream) {
  if (!in || !out || in == out || nb <= 0 || ph <= 0 || pw <= 0) return DC_ERR_ARG;
  const long total = (long)nb * ph * pw;
  hipLaunchKernelGGL(dilate_kernel, dim3((unsigned)min((total + 255) / 256, 65536L)), dim3(256), 0,
                     (hipStream_t)stream, in, ph, pw, total, out);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" long long dc_mask_rows_ws_bytes(long long total) { return ((total + kChunk - 1) / kChunk) * 4; }

// pass 1: count[0] = number of set pixels (ws: dc_mask_rows_ws_bytes)
extern "C" int dc_mask_count(const unsigned char* mask, long long total, int* ws, int* count, void* stream) {
  if (!mask || !ws || !count || total <= 0 || total > (1LL << 31) - 1) return DC_ERR_ARG;
  const int nchunk = (int)((total + kChunk - 1) / kChunk);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(chunk_count_kernel, dim3(nchunk), dim3(kChunk), 0, st, mask, (long)total, ws);
  hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(kChunk), 0, st, ws, nchunk, count);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// pass 2 (after dc_mask_count on the same mask / ws): rows[0..count) = sorted indices of the set pixels,
// rows[count..pad_to) = the last of them
extern "C" int dc_mask_rows(const unsigned char* mask, long long total, const int* ws, const int* count, int pad_to,
                            int* rows, void* stream) {
  if (!mask || !ws || !count || !rows || total <= 0 || pad_to < 0) return DC_ERR_ARG;
  const int nchunk = (int)((total + kChunk - 1) / kChunk);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(compact_kernel, dim3(nchunk), dim3(kChunk), 0, st, mask, (long)total, ws, rows);
  if (pad_to > 0)
    hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)min((pad_to + 255) / 256, 1024)), dim3(256), 0, st, rows,
                       count, pad_to);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// rows[count[0] .. pad_to) = the last listed pixel: the padding of dc_mask_rows(..., pad_to, ...) as its own launch,
// for hosts that list the rows before they know pad_to (the padded size waits for count[0] on the host)
extern "C" int dc_pad_rows(int* rows, const int* count, int pad_to, void* stream) {
  if (!rows || !count || pad_to < 0) return DC_ERR_ARG;
  if (pad_to == 0) return DC_OK;
  hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)min((pad_to + 255) / 256, 1024)), dim3(256), 0,
                     (hipStream_t)stream, rows, count, pad_to);
  DC_CHECK_LAUNCH();
  return DC_OK;
}
