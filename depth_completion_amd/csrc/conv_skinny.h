#pragma once
// Weight-streaming "skinny" conv / linear for the few-pixel layers of a batch-1 step (included after conv_gemm_impl.h,
// inside an anonymous namespace, by conv_gemm.hip for the variant table / contract and by conv_skinny9.hip /
// conv_skinny1.hip (and their fused-GroupNorm-statistics forms, conv_skinny{9,1}_gn.hip) for the kernels;
// dc_conv_gemm algo ids after the halo and im2col variants).
//
// UNet levels 2-3 at batch 1 have M = 432 / 108 output pixels against 1280-2560 channels: a 3x3 conv there reads
// 29.5 MB of weights for 3-13 GFLOP, so the launch is bound by how fast the weights stream from HBM (and, at
// M = 432, by MFMA), not by operand reuse.  The im2col / halo tiles stage the weights through an LDS ring shared
// by row tiles that each re-read them, and keep only a few KB per CU in flight.  Here a block owns ALL the pixels
// of its spatial tile (a whole level-3 frame, half or all of a level-2 frame, or a run of token rows) and
// 64 * NJ output channels; the four waves split the channels (16 * NJ each), so every weight byte is fetched by
// exactly one wave, straight into VGPRs (16 B per lane = one B fragment of v_mfma_f32_16x16x32_bf16, rows of the
// [cout][ktot] weight at the lane's output channel), one group ahead:
//   * a group is U input chunks of 64 channels x KT taps x 2 k-steps of 32 (G = 2 U KT k-steps); while group g
//     computes, each of its k-steps re-fills its register slot with the same k-step of group g + 1, so G NJ KB per
//     wave (18-36 KB for a 3x3 group) stay in flight -- enough to cover HBM latency at one block per CU;
//   * the activations of a group (KT 9: the (TH+2) x (TW+2) halo of the tile, halo rows padded to a multiple of 8
//     so that every tap's row offset is a compile-time immediate and keeps the XOR swizzle phase; KT 1: the tile's
//     rows) go into LDS by LDS-DMA one group ahead (double-buffered), with one barrier per group; all four waves
//     read them as the A fragments (ds_read_b128, conflict-free swizzle, per-lane addresses precomputed for the
//     three kx phases, the second k-step one XOR away).
// Input chunks split over blocks (split-K) are summed in split order, deterministically, either by the tile's
// last-arriving block (splitk > 0) or by a second kernel over (tile, fragment row) (splitk < 0); the epilogue stages
// the tile in LDS and writes 16-B rows.
// Contract (skinny_eligible): KT 9 = the halo contract (3x3, stride 1, pad 1, direct or nearest-upsample input,
// whole 64-channel chunks); KT 1 = 1x1 / linear over whole 64-channel chunks; no row list, no GEGLU; input chunks a
// multiple of U.  Fused GroupNorm statistics (dc_gn_fuse modes 1 / 2) ride in the epilogue that stores the tile: the
// unsplit / last-arriving block's, or skinny_reduce_kernel's.

template <int KT, int TH, int TW, int NJ, int U>
struct SkinnyCfg {
  static_assert(KT == 1 || KT == 9, "1x1 rows or 3x3 halo");
  static constexpr int BM = TH * TW;                       // output pixels of the tile
  static constexpr int MI = (BM + 15) / 16;
  static constexpr int BMP = MI * 16;
  static constexpr int BN = 64 * NJ, WN = 16 * NJ;
  static constexpr int W8 = KT == 9 ? ((TW + 2 + 7) / 8) * 8 : 1;   // halo row width, padded to a multiple of 8
  static constexpr int AROWS = KT == 9 ? (TH + 2) * W8 : BM;
  static constexpr int LA = (AROWS + 31) / 32;             // block-wide 16-B LDS-DMA instructions per chunk
  static constexpr int SLOT = LA * 32 * 128;               // one chunk's rows x 64 channels
  static constexpr int RING = 2 * U * SLOT;                // two groups
  static constexpr int G = U * KT * 2;                     // k-steps per group
  static constexpr int LDE = BN + 8;
  static constexpr int EPI = BMP * LDE * 2;                // block-wide bf16 staging tile
  static constexpr int LDS = RING > EPI ? RING : EPI;
  static constexpr int NA = KT == 9 ? 3 : 1;               // precomputed A addresses per fragment (kx phases)
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(G * NJ + U * LA <= 63, "vmcnt range");
  static_assert(KT == 1 || W8 * 128 * 2 + 2 * 128 < 65536, "tap offsets as ds_read immediates");
};

template <int KT, int TH, int TW, int NJ, int U, int GNM>
struct SkinnyBlock {
  using C = SkinnyCfg<KT, TH, TW, NJ, U>;
  static constexpr int MI = C::MI, G = C::G, LA = C::LA, NA = C::NA;
  static constexpr int kOOB = (int)0x80000000u;

  const ConvGemmParams& p;
  char* smem;
  int lane, wid_s;
  int frame, oy0, ox0, n0;
  long m0;
  int a_off[LA], a_off2[LA];
  int w_off[NJ];
  int ab[MI][NA];   // per-lane LDS byte address of each A fragment (tap (0, kx), first k-step)
  __amdgpu_buffer_rsrc_t ra, ra2, rb;
  f32x4 acc[MI][NJ];
  bf16x8 wr[G][NJ];

  // LDS-DMA of input chunk c (64 channels) into A slot `slot` (dead: out-of-range sources, zero-filled into a slot
  // nobody reads again, so that every group issues the same loads and the vmcnt accounting stays static)
  __device__ __forceinline__ void issue_a(int c, int slot, bool live) {
    DC_LDS char* b = (DC_LDS char*)smem + slot * C::SLOT;
    const int ch = c * 64;
    if (ch >= p.c1) {
#pragma unroll
      for (int j = 0; j < LA; ++j)
        buf_load_lds16(ra2, b + (wid_s * 64 + 256 * j) * 16, live ? a_off2[j] : kOOB, (ch - p.c1) * 2);
    } else {
#pragma unroll
      for (int j = 0; j < LA; ++j)
        buf_load_lds16(ra, b + (wid_s * 64 + 256 * j) * 16, live ? a_off[j] : kOOB, ch * 2);
    }
  }

  // B fragments of k-step S of the group whose first input chunk is cg; wv: the lanes' weight-row offsets (kOOB for
  // the dead loads after the last group: zero, no traffic)
  template <int S>
  __device__ __forceinline__ void load_w(int cg, const int (&wv)[NJ]) {
    constexpr int J = S / (2 * KT), T = (S / 2) % KT, H = S % 2;
    const int soff = (T * p.cin + (cg + J) * 64 + H * 32) * 2;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      // default cache policy: nt (aux 2) measured 2.2 % slower at C2 (profiles/r06b/)
      const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rb, wv[jj], soff, 0);
      wr[S][jj] = __builtin_bit_cast(bf16x8, v);
    }
  }

  // The group's MFMA work as L = G x MI fragment steps (k-step F / MI, pixel fragment F % MI): step F runs the NJ
  // MFMAs of its A fragment and issues the LDS read of fragment F + D (a D-deep register ring keeps the LDS latency
  // under D steps of MFMAs); the last fragment of a k-step re-fills that k-step's weight registers for the next group.
  static constexpr int L = G * MI;
  static constexpr int D = (NJ == 1 ? 8 : 6) < L ? (NJ == 1 ? 8 : 6) : L;
  template <int F>
  __device__ __forceinline__ void read_frag(bf16x8 (&af)[D]) {
    constexpr int S = F / MI, II = F % MI;
    constexpr int J = S / (2 * KT), T = (S / 2) % KT, H = S % 2;
    constexpr int KY = KT == 9 ? T / 3 : 0, KX = KT == 9 ? T % 3 : 0;
    constexpr int IMM = J * C::SLOT + KY * C::W8 * 128;
    const int a = H ? (ab[II][KX] ^ 64) : ab[II][KX];
    af[F % D] = *reinterpret_cast<const bf16x8*>(smem + a + IMM);
  }
  template <int F>
  __device__ __forceinline__ void frag_step(bf16x8 (&af)[D], int cgn, const int (&wv)[NJ]) {
    constexpr int S = F / MI, II = F % MI;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj)
      acc[II][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[F % D], wr[S][jj], acc[II][jj], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, NJ, 0);
    if constexpr (F + D < L) {
      read_frag<F + D>(af);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if constexpr (II == MI - 1) {
      // pinned here (no memory operation crosses the asm): the compiler otherwise sinks every load of the group to
      // its end, and then the next group's first MFMA waits for all of them
      load_w<S>(cgn, wv);
      asm volatile("" ::: "memory");
    }
  }
  template <int... P>
  __device__ __forceinline__ void read_first(bf16x8 (&af)[D], std::integer_sequence<int, P...>) {
    (read_frag<P>(af), ...);
  }
  template <int... F>
  __device__ __forceinline__ void group(int cgn, const int (&wv)[NJ], std::integer_sequence<int, F...>) {
    bf16x8 af[D];
    read_first(af, std::make_integer_sequence<int, D>{});
    __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
    (frag_step<F>(af, cgn, wv), ...);
  }
  template <int S>
  __device__ __forceinline__ void load_pinned(int cg, const int (&wv)[NJ]) {
    load_w<S>(cg, wv);
    asm volatile("" ::: "memory");
  }
  // the prologue's loads in k-step order, as the loop issues them (the vmcnt counts at the loop head merge both paths)
  template <int... S>
  __device__ __forceinline__ void load_group(int cg, const int (&wv)[NJ], std::integer_sequence<int, S...>) {
    (load_pinned<S>(cg, wv), ...);
  }

  __device__ __forceinline__ void run() {
    const int tid = threadIdx.x;
    lane = tid & 63;
    wid_s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wid = tid >> 6;
    // ---- block -> (split, column tile, spatial tile): split-major; within a split the spatial tiles of a column
    // tile are adjacent (they read the same weight slice, on the same XCD)
    const int tiles_n = (p.cout + C::BN - 1) / C::BN;
    const int tiles = gridDim.x, nblk = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int wk = xcd_remap(bid, nblk);
    const int split = wk / tiles;
    const int lb = wk - split * tiles;
    const int tiles_sp = tiles / tiles_n;
    const int tn = lb / tiles_sp, sp = lb - tn * tiles_sp;
    n0 = tn * C::BN;
    const long M = conv_rows(p);
    if constexpr (KT == 9) {
      const int tiles_x = (p.wout + TW - 1) / TW, tiles_y = (p.hout + TH - 1) / TH;
      frame = sp / (tiles_y * tiles_x);
      const int trem = sp - frame * (tiles_y * tiles_x);
      oy0 = (trem / tiles_x) * TH;
      ox0 = (trem - (trem / tiles_x) * tiles_x) * TW;
      m0 = 0;
    } else {
      frame = oy0 = ox0 = 0;
      m0 = (long)sp * TH;
    }
    const int nck = p.cin / 64;
    const int c_begin = __builtin_amdgcn_readfirstlane(split * p.kps);
    const int c_end = min(nck, c_begin + p.kps);
    const int ngr = max(0, c_end - c_begin) / U;

    // ---- per-lane LDS-DMA source offsets of the A rows (the chunk's channel offset rides in soffset)
    const int slot = tid & 7, r0 = tid >> 3;
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      const int hr = r0 + 32 * j;
      bool ok;
      long pix;
      if constexpr (KT == 9) {
        const int hy = hr / C::W8, hx = hr - (hr / C::W8) * C::W8;
        const int vy = oy0 - 1 + hy, vx = ox0 - 1 + hx;
        ok = hr < C::AROWS && hx < TW + 2 && vy >= 0 && vy < p.hout && vx >= 0 && vx < p.wout;
        int iy = vy, ix = vx;
        if (p.mode == 1) {
          iy = ok ? (int)fast_div((unsigned)(vy * p.hin), p.h_mul, p.h_shr) : 0;
          ix = ok ? (int)fast_div((unsigned)(vx * p.win), p.w_mul, p.w_shr) : 0;
        }
        pix = ((long)frame * p.hin + iy) * p.win + ix;
      } else {
        pix = m0 + hr;
        ok = hr < C::AROWS && pix < M;
      }
      const int sw = (slot ^ (hr & 7)) * 8;
      a_off[j] = ok ? (int)((pix * p.ldx + sw) * 2) : kOOB;
      a_off2[j] = ok ? (int)((pix * p.ldx2 + sw) * 2) : kOOB;
    }
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int co = n0 + wid * C::WN + jj * 16 + (lane & 15);
      w_off[jj] = co < p.cout ? (co * p.ktot + 8 * (lane >> 4)) * 2 : kOOB;
    }
    ra = buf_rsrc(p.x);
    ra2 = buf_rsrc(p.x2);
    rb = buf_rsrc(p.w);
    // A fragment addresses (group 0's slots): row r of the tap-(0, kx) read, chunk (lane >> 4) of the first k-step
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      int pl = ii * 16 + (lane & 15);
      pl = pl < C::BM ? pl : 0;   // pad rows read a valid row; never stored
      const int rbase = KT == 9 ? (pl / TW) * C::W8 + (pl - (pl / TW) * TW) : pl;
#pragma unroll
      for (int kx = 0; kx < NA; ++kx) {
        const int r = rbase + kx;
        ab[ii][kx] = r * 128 + (((lane >> 4) ^ (r & 7)) << 4);
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (ngr > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) issue_a(c_begin + u, u, true);
      load_group(c_begin, w_off, std::make_integer_sequence<int, G>{});
    }
    for (int g = 0; g < ngr; ++g) {
      // the group's activations (older than its G NJ weight loads) have landed in every wave
      vm_wait<G * NJ>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int par = g & 1;
      const bool live = g + 1 < ngr;
      const int cgn = c_begin + (g + 1) * U;
#pragma unroll
      for (int u = 0; u < U; ++u) issue_a(cgn + u, (par ^ 1) * U + u, live);
      int wv[NJ];
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj) wv[jj] = live ? w_off[jj] : kOOB;
      group(cgn, wv, std::make_integer_sequence<int, L>{});
      // the next group reads the other half of the ring
      const int delta = par ? -U * C::SLOT : U * C::SLOT;
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int kx = 0; kx < NA; ++kx) ab[ii][kx] += delta;
    }
    vm_wait<0>();

    if (p.splits > 1) {
      if (p.sk_blocks < 0) {   // two-kernel form: the partial only; skinny_reduce_kernel sums and stores
        store_partial(lb, split, tiles);
        return;
      }
      if (!handoff(lb, split, tiles)) return;
    }
    epilogue(wid, M);
  }

  // ---- two-kernel split-K: this split's partial in the accumulator-native slab layout (the kernel boundary orders
  // it before skinny_reduce_kernel's reads)
  __device__ __forceinline__ void store_partial(int lb, int split, int tiles) {
    constexpr int FR = MI * NJ, WAVE_F = FR * 256, TILE_F = 4 * WAVE_F;
    const __amdgpu_buffer_rsrc_t rs = ws_rsrc(p.ws);
    const long mine = ((long)split * tiles + lb) * TILE_F + (threadIdx.x >> 6) * WAVE_F + lane * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) store_sc1_x4(rs, mine + (i * NJ + j) * 256, acc[i][j]);
  }

  // ---- split-K hand-off (the protocol of tile_handoff_g: sc1 partial stores, agent-scope arrival counter, the
  // last-arriving block sums every split's partial in split order).  The last arriver's read is latency-bound: a
  // skinny tile holds MI x NJ fragments per lane and the splits are many, so RS whole splits' partials (up to ~40
  // 16-B loads per lane) go out per round instead of one fragment row at a time.
  __device__ __forceinline__ bool handoff(int lb, int split, int tiles) {
    constexpr int FR = MI * NJ;                 // 16-B fragments per lane
    constexpr int WAVE_F = FR * 256, TILE_F = 4 * WAVE_F;
    constexpr int RS = FR >= 40 ? 1 : 40 / FR;  // splits per read round
    const int tid = threadIdx.x, wid = tid >> 6;
    const __amdgpu_buffer_rsrc_t rs = ws_rsrc(p.ws);
    const long mine = ((long)split * tiles + lb) * TILE_F + wid * WAVE_F + lane * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) store_sc1_x4(rs, mine + (i * NJ + j) * 256, acc[i][j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* s_last = reinterpret_cast<int*>(smem);
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + lb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_last = old == p.splits - 1;
    }
    __syncthreads();
    if (!*s_last) return false;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < p.splits; s0 += RS) {
      f32x4 part[RS][FR];
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        if (s0 + r < p.splits) {
          const long src = ((long)(s0 + r) * tiles + lb) * TILE_F + wid * WAVE_F + lane * 4;
#pragma unroll
          for (int f = 0; f < FR; ++f) part[r][f] = load_sc1_x4(rs, src + f * 256);
        }
      }
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        if (s0 + r < p.splits) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] += part[r][i * NJ + j];
        }
      }
    }
    if (tid == 0) p.counters[lb] = 0;   // ready for the next launch (ordered by the kernel boundary)
    return true;
  }

  // ---- epilogue: bias in fp32, the block's tile staged as bf16 in LDS, then 16-B rows of BN channels per pixel
  // (GNM: with the fused GroupNorm statistics of the stored rows, GnTileSums)
  __device__ __forceinline__ void epilogue(int wid, long M) {
    const int col_l = lane & 15, row_l = (lane >> 4) * 4;
    __syncthreads();
    bf16* es = reinterpret_cast<bf16*>(smem);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wid * C::WN + j * 16 + col_l;
      const int c = n0 + cl;
      const float bv = (p.bias && c < p.cout) ? p.bias[c] : 0.0f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) es[(i * 16 + row_l + q) * C::LDE + cl] = (bf16)(acc[i][j][q] + bv);
    }
    __syncthreads();
    if (p.diag & 64) return;   // experiments only: no epilogue stores
    constexpr int GPR = C::BN / 8;
    GnTileSums<GNM, GPR> gs;
    if constexpr (GNM != 0) gs.init(p, n0 + (int)(threadIdx.x % GPR) * 8);
    for (int g = threadIdx.x; g < C::BM * GPR; g += 256) {
      const int pl = g / GPR, cg = g - (g / GPR) * GPR;
      const int c = n0 + cg * 8;
      if (c >= p.cout) continue;
      long m;
      if constexpr (KT == 9) {
        const int oy = oy0 + pl / TW, ox = ox0 + (pl - (pl / TW) * TW);
        if (oy >= p.hout || ox >= p.wout) continue;
        m = ((long)frame * p.hout + oy) * p.wout + ox;
      } else {
        m = m0 + pl;
        if (m >= M) continue;
      }
      float v[8];
      load8(es + pl * C::LDE + cg * 8, v);
      if constexpr (GNM != 0) {
        epilogue_values8(p, m, c, v);
        gs.add(p, m, KT == 9 ? frame : (int)fast_div((unsigned)m, p.gn.t[0].hw_mul, p.gn.t[0].hw_shr), v);
        store8(p.y + m * p.ldy + c, v);
      } else {
        epilogue_store(p, m, c, v, false);
      }
    }
    if constexpr (GNM != 0) {
      // a halo tile lies in one frame; a row tile [m0, min(m0 + BM, M)) may run across frames
      int fa = frame, fb = frame;
      if constexpr (KT == 1) {
        const long last = min(m0 + C::BM, M) - 1;
        fa = (int)fast_div((unsigned)m0, p.gn.t[0].hw_mul, p.gn.t[0].hw_shr);
        fb = (int)fast_div((unsigned)last, p.gn.t[0].hw_mul, p.gn.t[0].hw_shr);
      }
      gs.template finish<C::BN>(p, reinterpret_cast<float*>(smem), n0, fa == fb, fa);
    }
  }
};

template <int KT, int TH, int TW, int NJ, int U, int GNM>
__global__ __launch_bounds__(256) void conv_skinny_kernel(const ConvGemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[SkinnyCfg<KT, TH, TW, NJ, U>::LDS];
  static_assert(GNM == 0 || SkinnyCfg<KT, TH, TW, NJ, U>::LDS >= (256 * 16 + 2 * 64 * NJ) * 4, "GroupNorm-sum LDS");
  SkinnyBlock<KT, TH, TW, NJ, U, GNM> blk{p, smem};
  blk.run();
}

// Two-kernel split-K (splitk < 0): the last-arriving block of a skinny tile would read every split's partial alone
// (splits x BMP x BN x 4 bytes through one CU, latency- and per-CU-bandwidth-bound); here one block per (tile, 16-pixel
// fragment row) sums that row's partials in split order (deterministic), adds the bias and runs the epilogue (GNM:
// with the fused GroupNorm statistics of its 16 rows, GnTileSums).
template <int KT, int TH, int TW, int NJ, int U, int GNM>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(const ConvGemmParams p) {
  using C = SkinnyCfg<KT, TH, TW, NJ, U>;
  constexpr int FR = C::MI * NJ, WAVE_F = FR * 256, TILE_F = 4 * WAVE_F;
  __shared__ __attribute__((aligned(16))) bf16 es[16 * C::LDE];
  __shared__ __attribute__((aligned(16))) float red[GNM ? 256 * 16 + 2 * C::BN : 1];
  const int lb = blockIdx.x, ii = blockIdx.y, tiles = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = (p.cout + C::BN - 1) / C::BN, tiles_sp = tiles / tiles_n;
  const int tn = lb / tiles_sp, sp = lb - tn * tiles_sp;
  const int n0 = tn * C::BN;
  const __amdgpu_buffer_rsrc_t rs = ws_rsrc(p.ws);
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  // every split's partial of the lane's NJ fragments in flight at once (rounds of RK loads), summed in split order
  constexpr int RK = 16;
  f32x4 s[NJ];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) s[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long base = (long)lb * TILE_F + wid * WAVE_F + ii * NJ * 256 + lane * 4;
  for (int k0 = 0; k0 < p.splits; k0 += RK) {
    f32x4 part[RK][NJ];
#pragma unroll
    for (int k = 0; k < RK; ++k)
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj)
        if (k0 + k < p.splits) part[k][jj] = load_sc1_x4(rs, base + (long)(k0 + k) * tiles * TILE_F + jj * 256);
#pragma unroll
    for (int k = 0; k < RK; ++k)
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj)
        if (k0 + k < p.splits) s[jj] += part[k][jj];
  }
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int cl = wid * C::WN + jj * 16 + col_l;
    const int c = n0 + cl;
    const float bv = (p.bias && c < p.cout) ? p.bias[c] : 0.0f;
#pragma unroll
    for (int e = 0; e < 4; ++e) es[(row_l + e) * C::LDE + cl] = (bf16)(s[jj][e] + bv);
  }
  __syncthreads();
  if (p.diag & 64) return;
  constexpr int GPR = C::BN / 8;
  const long M = conv_rows(p);
  int frame = 0;
  if constexpr (KT == 9) {
    const int tiles_x = (p.wout + TW - 1) / TW, tiles_y = (p.hout + TH - 1) / TH;
    frame = sp / (tiles_y * tiles_x);
  }
  GnTileSums<GNM, GPR> gs;
  if constexpr (GNM != 0) gs.init(p, n0 + (tid % GPR) * 8);
  for (int g = tid; g < 16 * GPR; g += 256) {
    const int r = g / GPR, cg = g - (g / GPR) * GPR;
    const int pl = ii * 16 + r;
    const int c = n0 + cg * 8;
    if (pl >= C::BM || c >= p.cout) continue;
    long m;
    if constexpr (KT == 9) {
      const int tiles_x = (p.wout + TW - 1) / TW, tiles_y = (p.hout + TH - 1) / TH;
      const int trem = sp - frame * (tiles_y * tiles_x);
      const int oy = (trem / tiles_x) * TH + pl / TW, ox = (trem - (trem / tiles_x) * tiles_x) * TW + pl % TW;
      if (oy >= p.hout || ox >= p.wout) continue;
      m = ((long)frame * p.hout + oy) * p.wout + ox;
    } else {
      m = (long)sp * TH + pl;
      if (m >= M) continue;
    }
    float v[8];
    load8(es + r * C::LDE + cg * 8, v);
    if constexpr (GNM != 0) {
      epilogue_values8(p, m, c, v);
      gs.add(p, m, KT == 9 ? frame : (int)fast_div((unsigned)m, p.gn.t[0].hw_mul, p.gn.t[0].hw_shr), v);
      store8(p.y + m * p.ldy + c, v);
    } else {
      epilogue_store(p, m, c, v, false);
    }
  }
  if constexpr (GNM != 0) {
    // the 16 rows' frames (a halo tile lies in one frame; token rows may run across frames)
    int fa = frame, fb = frame;
    if constexpr (KT == 1) {
      const long first = (long)sp * TH + ii * 16;
      // a trailing 16-row fragment of the last tile can start past the last row (M = 108 on 128-row tiles): it stored
      // nothing, so it adds nothing -- return (block-uniform) rather than form a frame index past the last frame
      if (first >= M) return;
      const long last = min(min(first + 16, (long)sp * TH + C::BM), M) - 1;
      fa = (int)fast_div((unsigned)first, p.gn.t[0].hw_mul, p.gn.t[0].hw_shr);
      fb = (int)fast_div((unsigned)max(last, first), p.gn.t[0].hw_mul, p.gn.t[0].hw_shr);
    }
    gs.template finish<C::BN>(p, red, n0, fa == fb, fa);
  }
}

// skinny variants: taps (9: halo tile TH x TW of one frame; 1: TH token / pixel rows), NJ x 64 output channels per
// block, U input chunks per group
struct SkinnyAlgo {
  int kt, th, tw, nj, u;
};
constexpr SkinnyAlgo kSkinnyAlgos[] = {
    {9, 9, 12, 1, 1},    // level 3 frame (108 px) x 64 (48 KB LDS)
    {9, 9, 12, 2, 1},    // level 3 frame x 128
    {9, 9, 24, 1, 1},    // half a level-2 frame (216 px) x 64 (88 KB)
    {9, 6, 24, 2, 1},    // a third of a level-2 frame (144 px) x 128 (64 KB)
    {9, 6, 24, 1, 1},    // a third of a level-2 frame x 64
    {1, 112, 1, 1, 4},   // 112 rows x 64, 4-chunk groups (128 KB)
    {1, 112, 1, 2, 2},   // 112 rows x 128, 2-chunk groups (64 KB)
    {1, 112, 1, 2, 4},   // 112 rows x 128, 4-chunk groups (128 KB)
    {1, 224, 1, 1, 2},   // 224 rows x 64 (112 KB)
    {1, 224, 1, 2, 2},   // 224 rows x 128 (112 KB)
    {1, 64, 1, 2, 4},    // 64 rows x 128 (64 KB)
    {1, 144, 1, 2, 2},   // 144 rows x 128 (72 KB)
};
constexpr int kNumSkinny = sizeof(kSkinnyAlgos) / sizeof(kSkinnyAlgos[0]);

bool skinny_eligible(const ConvGemmParams& p, int i) {
  if (i < 0 || i >= kNumSkinny || p.rows || p.geglu) return false;
  const SkinnyAlgo& a = kSkinnyAlgos[i];
  if (p.cin % 64 != 0 || (p.cin / 64) % a.u != 0) return false;
  if (p.c1 < p.cin && p.c1 % 64 != 0) return false;
  if ((long)p.cout * p.ktot * 2 >= (1L << 31)) return false;
  const long ld = p.ldx > p.ldx2 ? p.ldx : p.ldx2;
  if ((long)p.nb * p.hin * p.win * ld * 2 >= (1L << 31)) return false;
  if (a.kt == 9) return halo_eligible(p);
  return p.kh == 1 && p.kw == 1 && p.stride == 1 && p.pad == 0 && p.mode == 0 && p.hin == p.hout &&
         p.win == p.wout && p.ktot == p.cin;
}

template <int KT, int TH, int TW, int NJ, int U, int GNM>
int launch_skinny(ConvGemmParams& p, int splits, hipStream_t stream) {
  using Cf = SkinnyCfg<KT, TH, TW, NJ, U>;
  const long M = (long)p.nb * p.hout * p.wout;
  const long sp = KT == 9 ? (long)p.nb * ((p.hout + TH - 1) / TH) * ((p.wout + TW - 1) / TW) : (M + TH - 1) / TH;
  const long tiles_l = sp * ((p.cout + Cf::BN - 1) / Cf::BN);
  if (tiles_l >= (1L << 30)) return DC_ERR_ARG;
  const int tiles = (int)tiles_l;
  const int ngr = (p.cin / 64) / U;
  p.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(p.ws) + (p.ws_bytes - kCounterBytes));
  const bool sep = splits < 0;          // two-kernel split-K (skinny_reduce_kernel)
  splits = max(1, min(sep ? -splits : splits, ngr));
  if (p.ws == nullptr || tiles > kMaxSplitTiles) splits = 1;
  while (splits > 1 && (long)splits * tiles * Cf::BMP * Cf::BN * 4 > p.ws_bytes - kCounterBytes) --splits;
  const int gps = (ngr + splits - 1) / splits;   // groups per split
  splits = (ngr + gps - 1) / gps;
  p.kps = gps * U;
  p.splits = splits;
  p.sk_blocks = (sep && splits > 1) ? -1 : 0;
  hipLaunchKernelGGL((conv_skinny_kernel<KT, TH, TW, NJ, U, GNM>), dim3(tiles, splits), dim3(256), 0, stream, p);
  DC_CHECK_LAUNCH();
  if (p.sk_blocks < 0) {
    hipLaunchKernelGGL((skinny_reduce_kernel<KT, TH, TW, NJ, U, GNM>), dim3(tiles, Cf::MI), dim3(256), 0, stream, p);
    DC_CHECK_LAUNCH();
  }
  return DC_OK;
}

// launch of variant i, for the variants with KT taps (conv_skinny9.hip / conv_skinny1.hip instantiate them; the
// fused GroupNorm-statistics forms GNM 1 / 2 in conv_skinny{9,1}_gn.hip)
template <int KT, int GNM>
int launch_skinny_idx(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  switch (i) {
#define DC_SKINNY(i)                                                                                         \
  case i:                                                                                                    \
    if constexpr (kSkinnyAlgos[i].kt == KT)                                                                  \
      return launch_skinny<kSkinnyAlgos[i].kt, kSkinnyAlgos[i].th, kSkinnyAlgos[i].tw, kSkinnyAlgos[i].nj,   \
                           kSkinnyAlgos[i].u, GNM>(p, splits, s);                                            \
    return DC_ERR_ARG;
    DC_SKINNY(0) DC_SKINNY(1) DC_SKINNY(2) DC_SKINNY(3) DC_SKINNY(4) DC_SKINNY(5) DC_SKINNY(6) DC_SKINNY(7)
    DC_SKINNY(8) DC_SKINNY(9) DC_SKINNY(10) DC_SKINNY(11)
#undef DC_SKINNY
    default: return DC_ERR_ARG;
  }
}

// ---------------------------------------------------------------------------------------------------------
// Weight-resident persistent 3x3 conv for the narrow layers (cin = 64, cout <= 64: the TAESD encoder / decoder convs
// and their input gradients, every guided step at up to 288 x 384).  A 64 x 576 weight is 72 KB: each wave keeps its
// 16 output channels' 18 B fragments in VGPRs for the whole launch, and a block walks tiles t = blockIdx.x, +gridDim.x
// with the (TH+2) x (TW+2) halo of the next tile in flight (LDS-DMA into the other of two slots) while the current tile
// runs its 9 taps; the epilogue stages the tile in its own LDS region.  Per tile that leaves one barrier and the
// previous tile's stores left in flight (a static store count per tile, so the tile head waits only for its halo).  The halo-tile kernel (conv_halo_kernel) pays the weight ring's fill and its drain per tile.
template <int TH, int TW>
struct ResidentBlock {
  using C = SkinnyCfg<9, TH, TW, 1, 1>;   // halo geometry; 64 output channels (16 per wave); one 64-channel chunk
  static constexpr int MI = C::MI, G = C::G, LA = C::LA;
  static constexpr int L = G * MI;
  static constexpr int D = 8 < L ? 8 : L;
  static constexpr int ES = C::RING;                 // epilogue staging after the two halo slots
  static constexpr int LDS = C::RING + C::EPI;
  static constexpr int kOOB = (int)0x80000000u;
  static_assert(C::SLOT + 2 * C::W8 * 128 + 2 * 128 < 65536, "slot and tap offsets as ds_read immediates");
  static_assert(LDS <= 160 * 1024, "LDS");

  const ConvGemmParams& p;
  char* smem;
  int lane, wid_s, tiles_x, tiles_y;
  int ab[MI][3];
  __amdgpu_buffer_rsrc_t ra, rb;
  f32x4 acc[MI];
  bf16x8 wr[G];

  __device__ __forceinline__ void coords(int t, int& frame, int& oy0, int& ox0) const {
    frame = t / (tiles_y * tiles_x);
    const int r = t - frame * (tiles_y * tiles_x);
    oy0 = (r / tiles_x) * TH;
    ox0 = (r - (r / tiles_x) * tiles_x) * TW;
  }
  __device__ __forceinline__ void issue_halo(int t, int slot) {
    int frame, oy0, ox0;
    coords(t, frame, oy0, ox0);
    const int tid = threadIdx.x, sl = tid & 7, r0 = tid >> 3;
    DC_LDS char* b = (DC_LDS char*)smem + slot * C::SLOT;
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      const int hr = r0 + 32 * j;
      const int hy = hr / C::W8, hx = hr - (hr / C::W8) * C::W8;
      const int vy = oy0 - 1 + hy, vx = ox0 - 1 + hx;
      const bool ok = hr < C::AROWS && hx < TW + 2 && vy >= 0 && vy < p.hout && vx >= 0 && vx < p.wout;
      int iy = vy, ix = vx;
      if (p.mode == 1) {
        iy = ok ? (int)fast_div((unsigned)(vy * p.hin), p.h_mul, p.h_shr) : 0;
        ix = ok ? (int)fast_div((unsigned)(vx * p.win), p.w_mul, p.w_shr) : 0;
      }
      const long pix = ((long)frame * p.hin + iy) * p.win + ix;
      const int off = ok ? (int)((pix * p.ldx + (sl ^ (hr & 7)) * 8) * 2) : kOOB;
      buf_load_lds16(ra, b + (wid_s * 64 + 256 * j) * 16, off, 0);
    }
  }
  template <int PAR, int F>
  __device__ __forceinline__ void read_frag(bf16x8 (&af)[D]) {
    constexpr int S = F / MI, II = F % MI;
    constexpr int T = S / 2, H = S % 2, KY = T / 3, KX = T % 3;
    constexpr int IMM = PAR * C::SLOT + KY * C::W8 * 128;
    const int a = H ? (ab[II][KX] ^ 64) : ab[II][KX];
    af[F % D] = *reinterpret_cast<const bf16x8*>(smem + a + IMM);
  }
  template <int PAR, int F>
  __device__ __forceinline__ void frag_step(bf16x8 (&af)[D]) {
    constexpr int S = F / MI, II = F % MI;
    acc[II] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[F % D], wr[S], acc[II], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if constexpr (F + D < L) {
      read_frag<PAR, F + D>(af);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  }
  template <int PAR, int... P>
  __device__ __forceinline__ void read_first(bf16x8 (&af)[D], std::integer_sequence<int, P...>) {
    (read_frag<PAR, P>(af), ...);
  }
  template <int PAR, int... F>
  __device__ __forceinline__ void compute(std::integer_sequence<int, F...>) {
    bf16x8 af[D];
    read_first<PAR>(af, std::make_integer_sequence<int, D>{});
    __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
    (frag_step<PAR, F>(af), ...);
  }

  // one tile: its halo (slot PAR) has landed after the wait; the next tile's goes into the other slot
  template <int PAR>
  __device__ __forceinline__ void tile(int t, int tnext, int tiles) {
    vm_wait<NIT>();   // this tile's halo; the previous tile's NIT stores (younger) may still be in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tnext < tiles) issue_halo(tnext, PAR ^ 1);
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    compute<PAR>(std::make_integer_sequence<int, L>{});
    epilogue(t);
  }

  // Exactly NIT 16-B stores per thread per tile (pixels outside the frame store out of range: dropped), so that the
  // next tile's head waits for its halo with a static vmcnt(NIT) and leaves this tile's stores in flight.
  static constexpr int NIT = C::BM * (C::BN / 8) / 256;
  static_assert(C::BM * (C::BN / 8) % 256 == 0, "whole store rounds");
  __device__ __forceinline__ void epilogue(int t) {
    int frame, oy0, ox0;
    coords(t, frame, oy0, ox0);
    const int wid = threadIdx.x >> 6;
    const int col_l = lane & 15, row_l = (lane >> 4) * 4;
    bf16* es = reinterpret_cast<bf16*>(smem + ES);
    const int cl = wid * 16 + col_l;
    const float bv = (p.bias && cl < p.cout) ? p.bias[cl] : 0.0f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) es[(i * 16 + row_l + q) * C::LDE + cl] = (bf16)(acc[i][q] + bv);
    __syncthreads();
    constexpr int GPR = C::BN / 8;
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(p.y);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int g = threadIdx.x + 256 * it;
      const int pl = g / GPR, cg = g - (g / GPR) * GPR;
      const int c = cg * 8;
      const int oy = oy0 + pl / TW, ox = ox0 + (pl - (pl / TW) * TW);
      const bool ok = c < p.cout && oy < p.hout && ox < p.wout && !(p.diag & 64);
      const long m = ok ? ((long)frame * p.hout + oy) * p.wout + ox : 0;
      float v[8];
      load8(es + pl * C::LDE + c, v);
      if (p.rowbias) {
        const bf16* rb = p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (ok ? (float)rb[i] : 0.0f);
      }
      if (p.resid && ok) {
        float rf[8];
        load8(p.resid + m * p.ldr + c, rf);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + rf[i];
      }
      if (p.act == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
      }
      if (p.mask && ok) {
        float mf[8];
        load8(p.mask + m * p.ldmask + c, mf);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = mf[i] > 0.0f ? v[i] : 0.0f;
      }
      bf16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, o), ry, ok ? (int)((m * p.ldy + c) * 2) : kOOB,
                                             0, 0);
    }
  }

  __device__ __forceinline__ void run() {
    const int tid = threadIdx.x;
    lane = tid & 63;
    wid_s = __builtin_amdgcn_readfirstlane(tid >> 6);
    tiles_x = (p.wout + TW - 1) / TW;
    tiles_y = (p.hout + TH - 1) / TH;
    const int tiles = p.nb * tiles_x * tiles_y;
    int t = blockIdx.x;
    const int step = gridDim.x;
    if (t >= tiles) return;
    ra = buf_rsrc(p.x);
    rb = buf_rsrc(p.w);
    // the wave's 16 output channels x 576 weights, once: B fragments of the 18 k-steps (tap T, half H)
    const int co = (tid >> 6) * 16 + (lane & 15);
    const int wo = co < p.cout ? (co * p.ktot + 8 * (lane >> 4)) * 2 : kOOB;
#pragma unroll
    for (int s = 0; s < G; ++s)
      wr[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, wo, ((s / 2) * 64 + (s % 2) * 32) * 2, 0));
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      int pl = ii * 16 + (lane & 15);
      pl = pl < C::BM ? pl : 0;
      const int rbase = (pl / TW) * C::W8 + (pl - (pl / TW) * TW);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int r = rbase + kx;
        ab[ii][kx] = r * 128 + (((lane >> 4) ^ (r & 7)) << 4);
      }
    }
    issue_halo(t, 0);
    vm_wait<0>();   // the weights and the first halo
    for (;;) {
      tile<0>(t, t + step, tiles);
      t += step;
      if (t >= tiles) break;
      tile<1>(t, t + step, tiles);
      t += step;
      if (t >= tiles) break;
    }
    vm_wait<0>();
  }
};

template <int TH, int TW>
__global__ __launch_bounds__(256) void conv_resident_kernel(const ConvGemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[ResidentBlock<TH, TW>::LDS];
  ResidentBlock<TH, TW> blk{p, smem};
  blk.run();
}

// resident variants (TH, TW): 8 x 16 (78 KB LDS, two blocks per CU), 8 x 32 (138 KB, one), 4 x 32 (78 KB), 4 x 16 (49 KB)
struct ResidentAlgo {
  int th, tw;
};
constexpr ResidentAlgo kResidentAlgos[] = {{8, 16}, {8, 32}, {4, 32}, {4, 16}};
constexpr int kNumResident = sizeof(kResidentAlgos) / sizeof(kResidentAlgos[0]);

bool resident_eligible(const ConvGemmParams& p) {
  return p.gn.mode == 0 && p.cin == 64 && p.cout <= 64 && p.cout % 8 == 0 && p.c1 >= p.cin && halo_eligible(p) &&
         (long)p.nb * p.hout * p.wout * p.ldy * 2 < (1L << 31);
}

// bpc: blocks per CU of the persistent grid (the dc_conv_desc split field; 0: as many as the LDS allows)
template <int TH, int TW>
int launch_resident(ConvGemmParams& p, int bpc, hipStream_t stream) {
  const long tiles_l = (long)p.nb * ((p.hout + TH - 1) / TH) * ((p.wout + TW - 1) / TW);
  if (tiles_l >= (1L << 30)) return DC_ERR_ARG;
  const int fit = (int)((160L * 1024) / ResidentBlock<TH, TW>::LDS);
  bpc = bpc <= 0 ? fit : min(bpc, fit);
  const int grid = (int)min(tiles_l, (long)bpc * 256);
  p.splits = 1;
  p.sk_blocks = 0;
  hipLaunchKernelGGL((conv_resident_kernel<TH, TW>), dim3(grid), dim3(256), 0, stream, p);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

int launch_resident_idx(int i, ConvGemmParams& p, int bpc, hipStream_t s) {
  switch (i) {
#define DC_RESIDENT(i) \
  case i: return launch_resident<kResidentAlgos[i].th, kResidentAlgos[i].tw>(p, bpc, s);
    DC_RESIDENT(0) DC_RESIDENT(1) DC_RESIDENT(2) DC_RESIDENT(3)
#undef DC_RESIDENT
    default: return DC_ERR_ARG;
  }
}
