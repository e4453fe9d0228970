// Wave-specialised fused BN-backward dgrad (round 6): the 1x1 stride-1 dgrads of the train step
// whose fused epilogue outweighs their GEMM -- the Bottleneck conv1 dgrads that add into the
// residual-stream gradient, K <= 256 (bf16) / 128 (fp32) -- as a persistent kernel whose
// workgroups run the GEMM of output tile i+1 on four "producer" waves while four "consumer" waves
// drain tile i's fused BatchNorm-backward epilogue.
//
// Why: in gemm16_kernel a workgroup runs its tile's MFMA phase and then its epilogue, one after
// the other.  The stall counters of the bf16 dgrad (profiles/r6/r6b/pmc_stall_c5/) put 56% of its
// wave cycles on s_waitcnt / barriers with MFMA busy 12%: the epilogue's global loads are the
// critical path and the MFMA phase does not overlap them.
//
// Layout of one workgroup (512 threads, one per CU, all 160 KB of LDS):
//   * waves 0-3, the producers (one per SIMD: waves w and w + 4 share one, scripts/probe/
//     simd_map.hip): the 128x128 tile as 2x2 waves of 64x64 -- gemm16_kernel's 4-wave 128x128
//     tile: the same LDS-DMA k-tile images, swizzle, fragment reads and MFMA order, so dx is
//     bit-identical to it -- over a ring of three k-tile stages that runs on across tiles; after
//     the tile's last k-tile they write the accumulators to the staging tile;
//   * waves 4-7, the consumers: the epilogue of LdsBnbwd with the same thread -> (row, 8 columns)
//     map (rows rsub + 16 j, j = 0..7) and the same summation order of the partials, so bn_part is
//     bit-identical to the 4-wave tile's too; each thread holds all 8 of its rows' operands in
//     flight and re-issues every slot for tile i+1 as soon as it has consumed tile i's row;
//   * every wave runs the same barrier sequence (each role its own loop, wave-uniform): per tile
//     nk k-tile barriers (the producers' stage hand-off; the consumers process 8 / NKC rows after
//     each group of nk / NKC of them), B1 (the producers are done with the tile's k-tiles, the
//     consumers with the staging tile), B2 (the staging tile holds the next tile, the consumers'
//     column sums are in the stage just freed); B1, B2 once more for the last tile.
//   * the work: XCD x (blockIdx & 7) owns a contiguous range of m-tiles; its 32 workgroups split
//     into N/128 n-lanes x 32/(N/128) m-lanes, so each workgroup keeps one n-tile (coefficients
//     loaded once) and the n-tiles of one m-tile -- which gather the same dy rows -- run side by
//     side on one L2.
// Measured (profiles/r6/dgrad_ws/): bf16 28x28 512<-128 0.523 -> 0.469 ms, 14x14 1024<-256 0.297
// -> 0.239 ms (4.6-4.9 TB/s of the step's own bytes); the MFMA-bound dgrads (fp32 K >= 256, the
// conv3 dgrads) stay on the engine's tiles: there the producers alone reach the same ~100 TF.
#pragma once

namespace tmrg {

#ifndef TMR_DGRAD_WS
#define TMR_DGRAD_WS 1
#endif
constexpr int WS_NWG = 256;   // workgroups: one per CU (8 XCDs x 32)
// timing experiments only (wrong results): 1 -- the consumers keep the barrier sequence but do no
// epilogue work; 2 -- the producers keep their loads and barriers but issue no MFMA
#ifndef TMR_WS_EXP
#define TMR_WS_EXP 0
#endif

// The workgroup barrier of this kernel: LDS writes retired, then a raw s_barrier -- never
// __syncthreads(), whose fence emits vmcnt(0) while an LDS-DMA is in flight (an LDS-DMA is a
// pending LDS write on the VM counter: cdna_hip_programming.md, "Pipelining across barriers") and
// would drain the producers' next k-tile at every k-tile barrier.  The empty asm statements keep
// the compiler from moving memory accesses across it (the intrinsic itself is not a memory
// barrier to LLVM).  LDS-DMA data is ordered for another wave's ds_read by the issuing wave's
// counted vmcnt before this barrier.
__device__ __forceinline__ void ws_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The epilogue variant is fixed at compile time -- ReLU mask MSK (1: z > 0, 2: y*scale+shift >
// 0, 3: bits), the beta operand BETA -- so every row issues the same loads and the compiler can
// count vmcnt exactly (with loads behind run-time flags it waits for all of them).  bf16 (EpiForm
// 1): y, z, the old gradient and g bf16; fp32 (EpiForm 2): y, the old gradient and g fp32.
template <int F32, int NKC, int MSK, int BETA>
__global__ __launch_bounds__(512) void dgrad_ws_kernel(const GemmArgs a) {
  constexpr bool BN16 = !F32, C16 = !F32, G16 = !F32;   // y / z, old gradient, g: bf16
  constexpr int BM = 128, BN = 128, NW = 4, WN = 2;
  constexpr uint32_t ES = F32 ? 4u : 2u;
  constexpr int EPC = 16 / ES, BK = 128 / ES;
  constexpr int TM = 2, TN = 2;
  constexpr int ABYTES = BM * 128, STAGE = 2 * ABYTES;   // A and B images of one k-tile
  constexpr int NIA = ABYTES / (1024 * NW);                // LDS-DMA pieces per wave per image
  constexpr int NST = 3;                                   // k-tile stages
  constexpr int LDC = BN;                                  // fp32 row of the staged tile
  constexpr int STG = BM * LDC * 4;
  constexpr int CG = BN / 8, RPP = 256 / CG, NR = BM / RPP;   // 16 column groups, 16 rows / pass
  constexpr int R = NR / NKC;                               // consumer rows per group
  static_assert(NR == 8 && R * NKC == NR, "consumer row groups");
  static_assert(RPP * BN * 8 <= STAGE, "the partial sums fit a stage");
  using Frag = typename std::conditional<F32 != 0, f32x4_t, bf16x8>::type;
  // 3 x 32 KB stages + the 64 KB staging tile: the whole 160 KB.  The staged tile is unpadded, its
  // 32-column halves swapped on rows with bit 2 set (the two row sets of one accumulator store hit
  // disjoint banks); the consumers' column sums go to the stage whose k-tile was the tile's last
  // (free from the producers' last MFMAs until they issue into it again after the next k-tile
  // barrier).
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NST * STAGE + STG];
  float* const stg = reinterpret_cast<float*>(smem + NST * STAGE);
  auto scol = [](int row, int c) { return c ^ (((row >> 2) & 1) << 5); };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // this workgroup's tiles: m-tiles mlo + ms + i * mstr (i < ntl) of n-tile nt
  const int nnt = a.N / BN;
  const int mt = (a.M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int mlo = (int)((long)mt * xcd / 8), mhi = (int)((long)mt * (xcd + 1) / 8);
  const int nt = slot % nnt, ms = slot / nnt, mstr = (WS_NWG / 8) / nnt;
  const int ntl = mhi - mlo > ms ? (mhi - mlo - ms + mstr - 1) / mstr : 0;
  const int n0 = nt * BN;
  const int nk = (a.K + BK - 1) / BK;
  const int kpg = nk / NKC;   // k-tiles per consumer group (the host checks nk % NKC == 0)

  if (wave < NW) {
    // ================================ producers ================================
    const int lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int l31 = lane & 31, hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.A, a.Abytes);
    const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.B, a.Bbytes);
    // piece q of this wave: image rows 8 * (wave + NW * q) + lane / 8, 16-B chunk (lane & 7) ^
    // ((row >> 1) & 7) (the engine's K-contiguous image)
    int prow[NIA], pch[NIA];
    uint32_t boff[NIA];
#pragma unroll
    for (int q = 0; q < NIA; ++q) {
      prow[q] = 8 * (wave + NW * q) + (lane >> 3);
      pch[q] = EPC * ((lane & 7) ^ ((prow[q] >> 1) & 7));
      boff[q] = (uint32_t)(n0 + prow[q]) * (uint32_t)a.ldbt * ES + (uint32_t)pch[q] * ES;
    }
    // k-tile kt of the tile at row m0 -> LDS stage buf (A: dy rows, B: Wt rows of the n-tile)
    // piece q of the A and of the B image
    auto stage_q = [&](int m0, int kt, int buf, int q) {
      const int kb = kt * BK;
      unsigned char* As = smem + buf * STAGE;
      unsigned char* Bs = As + ABYTES;
      const int m = m0 + prow[q];
      const bool ok = m < a.M && kb + pch[q] < a.K;
      const uint32_t off = (uint32_t)m * (uint32_t)a.lds * ES + (uint32_t)(kb + pch[q]) * ES;
      glds16(rA, As + 1024 * (wave + NW * q), ok ? off : OOB);
      const bool okb = kb + pch[q] < a.K;
      glds16(rB, Bs + 1024 * (wave + NW * q), okb ? boff[q] + (uint32_t)kb * ES : OOB);
    };
    auto stage = [&](int m0, int kt, int buf) {
#pragma unroll
      for (int q = 0; q < NIA; ++q) stage_q(m0, kt, buf, q);
    };
    const int kx = (l31 >> 1) & 7;
    const int arow0 = wm * (BM / 2) + l31;
    const int brow0 = wn * (BN / WN) + l31;
    auto frags = [&](int buf, int s, Frag (&av)[TM], Frag (&bv)[TN]) {
      const unsigned char* As = smem + buf * STAGE;
      const unsigned char* Bs = As + ABYTES;
      const int ch = (2 * s + hh) ^ kx;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = *reinterpret_cast<const Frag*>(As + (arow0 + 32 * i) * 128 + (ch << 4));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = *reinterpret_cast<const Frag*>(Bs + (brow0 + 32 * j) * 128 + (ch << 4));
    };
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto mfmas = [&](const Frag (&av)[TM], const Frag (&bv)[TN]) {
      if constexpr (TMR_WS_EXP == 2) {
        asm volatile("" ::"v"(av[0]), "v"(bv[0]), "v"(av[TM - 1]), "v"(bv[TN - 1]));
        return;
      }
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F32) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][t], bv[j][t], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
    };
    // global k-tile G of this workgroup = k-tile G % nk of its tile G / nk, in stage G % NST
    const int ng = ntl * nk;
    auto stage_g = [&](int G) {
      const int ti = G / nk;
      stage((mlo + ms + ti * mstr) * BM, G - ti * nk, G % NST);
    };

    if (ntl > 0) {
      stage_g(0);
      if (ng > 1) stage_g(1);
      int g = 0;   // k-tiles consumed so far
      for (int i = 0; i < ntl; ++i) {
        for (int kt = 0; kt < nk; ++kt) {
          // this wave's pieces of k-tile g landed (those of g + 1, issued after them, may not)
          if (g + 1 < ng)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIA) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          ws_barrier();   // every producer's pieces of k-tile g landed; stage (g + 2) % 3 free
          const int buf = g % NST;
          Frag a0[TM], b0[TN], a1[TM], b1[TN];
          frags(buf, 0, a0, b0);
          // (spreading these pieces over the four k-steps measured no faster, round 6)
          if (g + 2 < ng) stage_g(g + 2);
          frags(buf, 1, a1, b1);
          mfmas(a0, b0);
          frags(buf, 2, a0, b0);
          mfmas(a1, b1);
          frags(buf, 3, a1, b1);
          mfmas(a0, b0);
          mfmas(a1, b1);
          ++g;
        }
        ws_barrier();   // B1: the consumers are done with the staging buffer
#pragma unroll
        for (int i2 = 0; i2 < TM; ++i2)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = wm * (BM / 2) + 32 * i2 + (r & 3) + 8 * (r >> 2) + 4 * hh;
              stg[row * LDC + scol(row, wn * (BN / WN) + 32 * j + l31)] = acc[i2][j][r];
              acc[i2][j][r] = 0.f;
            }
        ws_barrier();   // B2: the staging buffer holds tile i
      }
    }
    ws_barrier();   // B1 and
    ws_barrier();   // B2 of the last tile's epilogue
    return;
  }

  // ================================ consumers ================================
  const int etid = tid - 64 * NW;
  const int cg = etid % CG, rsub = etid / CG;
  const int col = n0 + 8 * cg;   // < N (N a multiple of 128)
  float mu[8], bsc[8], bsh[8], cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = a.bn_mean[col + e];
    bsc[e] = MSK == 2 ? a.bn_sc[col + e] : 0.f;
    bsh[e] = MSK == 2 ? a.bn_sh[col + e] : (MSK == 0 ? 1.f : 0.f);
    cs[e] = 0.f;
    cq[e] = 0.f;
  }
  // Every access of the epilogue is a buffer access at a byte offset (OOB for rows past M: loads
  // read zeros, stores drop), with no branches: the compiler then counts vmcnt exactly across the
  // loop, so consuming row slot j waits for that slot's loads only, not for the slots re-issued
  // after it (with per-row branches it waited for every load in flight).  Extents: the dx-shaped
  // span of C (elements), in each tensor's element size (the host keeps a launch under 2 GiB).
  const uint32_t span = G16 ? a.Cbytes / 2u : a.Cbytes / 4u;
  constexpr uint32_t ey = BN16 ? 2u : 4u, eo = C16 ? 2u : 4u, ec = G16 ? 2u : 4u;
  auto rsrc = [](const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rY = rsrc(a.bn_y, span * ey);
  const __amdgpu_buffer_rsrc_t rZ = rsrc(a.bn_z ? (const void*)a.bn_z : (const void*)a.bn_y,
                                         MSK == 3 ? (span + 31u) / 32u * 4u : span * ey);
  const __amdgpu_buffer_rsrc_t rO = rsrc(a.Cold ? a.Cold : (const void*)a.C, span * eo);
  const __amdgpu_buffer_rsrc_t rC = rsrc(a.C, span * ec);
  auto ld16 = [](__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  };
  struct In {
    uint4 y0, y1, z0, z1, c0, c1;
    uint32_t bits;
    uint32_t off;   // element offset of the row's 8 columns
    bool ok;
  };
  In pf[NR];
  // the loads of row slot j of the tile at row m0
  auto issue = [&](int m0, int j, In& x, bool live) {
    const int row = m0 + rsub + j * RPP;
    x.ok = live && row < a.M;
    x.off = (uint32_t)row * (uint32_t)a.ldc + (uint32_t)col;
    const uint32_t o = x.off;
    x.y0 = ld16(rY, x.ok ? o * ey : OOB);
    if constexpr (!BN16) x.y1 = ld16(rY, x.ok ? o * ey + 16u : OOB);
    if constexpr (MSK == 1) {
      x.z0 = ld16(rZ, x.ok ? o * ey : OOB);
      if constexpr (!BN16) x.z1 = ld16(rZ, x.ok ? o * ey + 16u : OOB);
    }
    if constexpr (MSK == 3)
      x.bits = __builtin_amdgcn_raw_buffer_load_b32(rZ, x.ok ? (o >> 5) * 4u : OOB, 0, 0);
    if constexpr (BETA != 0) {
      x.c0 = ld16(rO, x.ok ? o * eo : OOB);
      if constexpr (!C16) x.c1 = ld16(rO, x.ok ? o * eo + 16u : OOB);
    }
  };
  // row slot j of the staged tile: beta, mask, store, partial sums (LdsBnbwd::run's arithmetic;
  // a row past M adds nothing)
  auto consume = [&](const In& x, int j) {
    float yv[8], zv[8], old[8];
    if constexpr (BN16) {
      const uint32_t yu[4] = {x.y0.x, x.y0.y, x.y0.z, x.y0.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        yv[2 * e] = __uint_as_float(yu[e] << 16);
        yv[2 * e + 1] = __uint_as_float(yu[e] & 0xffff0000u);
      }
      if constexpr (MSK == 1) {
        const uint32_t zu[4] = {x.z0.x, x.z0.y, x.z0.z, x.z0.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          zv[2 * e] = __uint_as_float(zu[e] << 16);
          zv[2 * e + 1] = __uint_as_float(zu[e] & 0xffff0000u);
        }
      }
    } else {
      const uint32_t yu[8] = {x.y0.x, x.y0.y, x.y0.z, x.y0.w, x.y1.x, x.y1.y, x.y1.z, x.y1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) yv[e] = __uint_as_float(yu[e]);
      if constexpr (MSK == 1) {
        const uint32_t zu[8] = {x.z0.x, x.z0.y, x.z0.z, x.z0.w, x.z1.x, x.z1.y, x.z1.z, x.z1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) zv[e] = __uint_as_float(zu[e]);
      }
    }
    if constexpr (MSK == 3) {
      const uint32_t b8 = x.bits >> (x.off & 31u);
#pragma unroll
      for (int e = 0; e < 8; ++e) zv[e] = ((b8 >> e) & 1u) ? 1.f : 0.f;
    } else if constexpr (MSK != 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) zv[e] = 0.f;
    }
    if constexpr (BETA != 0) {
      unpack_old8(x.c0, x.c1, old, C16);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) old[e] = 0.f;
    }
    const int rr = rsub + j * RPP;
    const float* srow = stg + rr * LDC + scol(rr, 8 * cg);
    const float4 a0 = *reinterpret_cast<const float4*>(srow);
    const float4 a1 = *reinterpret_cast<const float4*>(srow + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float tv = fmaf(a.beta, old[e], av[e]);
      const bool keep = zv[e] + fmaf(yv[e], bsc[e], bsh[e]) > 0.f;
      tv = keep ? tv : 0.f;
      if constexpr (G16) tv = bf16_rne(tv);
      v[e] = tv;
      const float s1 = cs[e] + tv, s2 = fmaf(tv, yv[e] - mu[e], cq[e]);
      cs[e] = x.ok ? s1 : cs[e];
      cq[e] = x.ok ? s2 : cq[e];
    }
    const uint32_t so = x.ok ? x.off * ec : OOB;
    if constexpr (G16) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (__float_as_uint(v[2 * e]) >> 16) | (__float_as_uint(v[2 * e + 1]) & 0xffff0000u);
      const u32x4_t q = {w[0], w[1], w[2], w[3]};
      __builtin_amdgcn_raw_buffer_store_b128(q, rC, so, 0, 0);
    } else {
      const u32x4_t q0 = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                          __float_as_uint(v[3])};
      const u32x4_t q1 = {__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                          __float_as_uint(v[7])};
      __builtin_amdgcn_raw_buffer_store_b128(q0, rC, so, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(q1, rC, x.ok ? so + 16u : OOB, 0, 0);
    }
  };
  // the tile's column sums: this thread's 8 columns -> red (between B1 and B2), in the stage of
  // k-tile `gl` (the tile's last); the sums over the RPP row slots -> bn_part row of m-tile mi
  // (after B2)
  float* red = nullptr;
  auto put_red = [&](int gl) {
    red = reinterpret_cast<float*>(smem + (gl % NST) * STAGE);   // [RPP][BN][2]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rsub * BN + 8 * cg + e) * 2] = cs[e];
      red[(rsub * BN + 8 * cg + e) * 2 + 1] = cq[e];
      cs[e] = 0.f;
      cq[e] = 0.f;
    }
  };
  auto finalize = [&](int mi) {
    if (etid < BN) {
      float t0 = 0.f, t1 = 0.f;
      for (int q = 0; q < RPP; ++q) {
        t0 += red[(q * BN + etid) * 2];
        t1 += red[(q * BN + etid) * 2 + 1];
      }
      a.bn_part[(long)mi * a.part_ld + n0 + etid] = make_float2(t0, t1);
    }
  };
  if (ntl > 0) {
    // tile 0: its rows' operands go in flight while the producers run its GEMM
#pragma unroll
    for (int j = 0; j < NR; ++j) issue((mlo + ms) * BM, j, pf[j], true);
    for (int kt = 0; kt < nk; ++kt) ws_barrier();
    ws_barrier();   // B1
    ws_barrier();   // B2: tile 0 staged
    // iteration i: tile i - 1 is staged; the loads of tile i go out as its rows are consumed
    // (i == ntl: the last tile, its GEMM barriers absent and its loads out of range -- the same
    // instructions, so the loop body and its vmcnt counts stay uniform)
    for (int i = 1; i <= ntl; ++i) {
      const bool more = i < ntl;
      const int m0 = (mlo + ms + i * mstr) * BM;
      const int kg = more ? kpg : 0;
#pragma unroll
      for (int jj = 0; jj < NKC; ++jj) {
        for (int u = 0; u < kg; ++u) ws_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = jj * R + r;
          if constexpr (TMR_WS_EXP == 1) continue;
          consume(pf[j], j);
          // (the scheduler would hoist the next row's loads over this row's use: both sets live)
          __builtin_amdgcn_sched_barrier(0);
          issue(m0, j, pf[j], more);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      ws_barrier();   // B1
      put_red(more ? (i + 1) * nk - 1 : i * nk - 1);   // (the k-tile the producers just finished)
      ws_barrier();   // B2: tile i staged (the last tile: the partials written)
      finalize(mlo + ms + (i - 1) * mstr);
    }
  } else {
    ws_barrier();   // the producers' last B1
    ws_barrier();   // and B2
  }

}

// The launch for a fused BN-backward dgrad, when its shape qualifies (else -1, nothing launched):
// 1x1, stride 1, no padding, one tap (dx row = dy row); the tile rules' 128-row tiles (so the
// partial rows are the ones the host counted); N a multiple of 128 with N / 128 dividing the 32
// workgroups of an XCD; whole k-tiles, 1, 2 or 4 of them (bf16 K <= 256, fp32 K <= 128: the
// epilogue-bound dgrads -- where the MFMA phase dominates, the engine's tiles do as well); enough
// tiles for 256 persistent workgroups; the train step's residual conv1 dgrad: bf16 -- mask from z,
// beta 1 on a bf16 old gradient, g stored bf16; fp32 -- mask bits, beta 1 on the fp32 old gradient.
// `a.io_tiles` (TMR_IO_TILES) keeps the one-tile-per-workgroup launch (the tests' comparison).
template <int F32>
int launch_dgrad_ws(const GemmArgs& a, int cfg, hipStream_t st) {
  static const int on = env_int("TMR_DGRAD_WS", TMR_DGRAD_WS);   // A/B of the kernel
  if (!on || a.io_tiles || a.bn_part == nullptr || a.pro) return -1;
  if (kCfgs16[cfg].bm != 128) return -1;
  if (a.ntaps != 1 || a.osy != 1 || a.osx != 1 || a.oyc != 0 || a.oxc != 0 || a.oy0 != 0 ||
      a.ox0 != 0 || a.wr0 != 0 || a.ws0 != 0 || a.sy != 1 || a.sx != 1 ||
      (long)a.Hs * a.Ws != (long)a.dHW.d || a.Ws != (int)a.dW.d || a.oH != a.Hs || a.oW != a.Ws)
    return -1;
  if (a.N % 128 != 0 || (WS_NWG / 8) % (a.N / 128) != 0) return -1;
  constexpr int bk = F32 ? 32 : 64;
  if (a.K <= 0 || a.K % bk != 0) return -1;
  const int nk = a.K / bk;
  if (cdiv(a.M, 128) * (long)(a.N / 128) < 2L * WS_NWG) return -1;
  const bool beta1 = a.beta == 1.f;
  const dim3 grid(WS_NWG), blk(512);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, blk, 0, st, a);
    TMR_CHECK_LAUNCH("dgrad_ws_kernel");
    __atomic_fetch_add(&g_dgrad_ws_launches, 1L, __ATOMIC_RELAXED);
    return 0;
  };
  if constexpr (F32) {
    // (K >= 256 and the conv3 dgrads are MFMA-bound: the four producer waves alone reach the
    // engine's ~100 TF and the epilogue traffic beside them costs 20-35%, so they stay on the
    // engine's tiles; profiles/r6/dgrad_ws/README.md)
    if (a.bn16 || a.g16 || a.cold16) return -1;
    static const int mfma_bound = env_int("TMR_DGRAD_WS_MFMA", 0);   // A/B of the wider scope
    if (a.bn_mask == 3 && beta1) {
      if (nk == 2) return go(dgrad_ws_kernel<1, 2, 3, 1>);
      if (nk == 4) return go(dgrad_ws_kernel<1, 4, 3, 1>);
      if (mfma_bound && nk % 8 == 0) return go(dgrad_ws_kernel<1, 8, 3, 1>);
    } else if (mfma_bound && a.bn_mask == 2 && a.beta == 0.f && nk % 8 == 0) {
      return go(dgrad_ws_kernel<1, 8, 2, 0>);
    }
  } else {
    if (!a.bn16 || !a.g16 || a.bn_mask != 1 || !beta1 || !(a.Cold == nullptr || a.cold16))
      return -1;
    if (nk == 1) return go(dgrad_ws_kernel<0, 1, 1, 1>);
    if (nk == 2) return go(dgrad_ws_kernel<0, 2, 1, 1>);
    if (nk == 4) return go(dgrad_ws_kernel<0, 4, 1, 1>);
  }
  return -1;
}

}  // namespace tmrg
