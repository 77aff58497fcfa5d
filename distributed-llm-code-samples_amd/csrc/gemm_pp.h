#pragma once
// bf16 256x128 MFMA GEMM with TWO blocks per CU ("ping-pong" by co-residency).  Included by gemm_kernels.h.
//
// Why: the 256x256 8-phase kernel holds one block per CU (128 KiB LDS), so while a block runs its epilogue (for
// the fused-SGD weight gradient: an fp32 master read-modify-write + a bf16 copy store, 10 B per parameter) no MFMA
// work is in flight on that CU, and a 224-tile TP shard grid leaves 32 CUs idle.  Here a block is 4 waves (one per
// SIMD) on a 256(M) x 128(N) output tile with 80 KiB of LDS, so two blocks share every CU: each SIMD carries one
// wave of each, and the hardware interleaves the two blocks' MFMA, LDS and memory segments with no barrier
// coupling between them.  One block's epilogue (or barrier wait) runs under the other's MFMAs: the wave-group
// ping-pong of a 2-consumer kernel, with the two groups in separate workgroups so neither waits for the other.
//
// Per wave: a 128x64 output piece as four 64x32 quadrant pieces (the 8-phase kernel's map, acc[2][2][4][2]), so
// the batched epilogues (act + ReLU bitmask, dact, glu, dglu, sgd, adam, store) are shared (epilogue_256, QNS 64).
//
// LDS (80 KiB): A half-tiles (128 rows x 64 k, 16 KiB) in a 3-slot ring, B half-tiles (64 cols x 64 k, 8 KiB) in
// 2 halves x 2 buffers.  Images as in the 8-phase kernel: K-contiguous [rows][64 k] with 16-B chunks XOR (row>>1)&7
// (ds_read_b128); MN-contiguous [64 k][mn] with 32-B units XOR-swizzled (ds_read_b64_tr_b16): 256-B rows for A
// (unit ^ mc_swz(k)), 128-B rows for B (unit ^ pp_swz(k)); all conflict-free, swizzles applied on the LDS-DMA
// source address (the DMA image is lane-linear).
//
// Schedule: 4 phases per 64-deep K-tile kk, phase q computes quadrant (0,0),(0,1),(1,1),(1,0) with 16 MFMAs per
// wave; one barrier per phase.  Reads: q0 A-h0 + B-h0, q1 B-h1, q2 A-h1, q3 none.  LDS-DMA, 3 x 1 KiB per wave per
// phase (A half = 4 pieces per wave, B half = 2):
//   q0: B1(kk+1)[1]  A0(kk+1)[2,3]        q1: A1(kk+1)[0,1]  B0(kk+2)[0]
//   q2: A1(kk+1)[2,3] B0(kk+2)[1]         q3: A0(kk+2)[0,1]  B1(kk+2)[0]
// A half j = 2kk + h goes to slot j % 3 (restaged >= 1 phase after its last read: A1(kk+1) reuses A0(kk)'s slot,
// A0(kk+2) A1(kk)'s); B halves to buffer kk & 1.  s_waitcnt vmcnt(9) at q1 and q3 retires everything issued up to
// 3 phases earlier: q1(kk) retires A1(kk) (read at q2), q3(kk) retires A0/B0/B1(kk+1) (read at q0/q1 of kk+1).
// Every piece has 3-4 phases of flight.  Each wave waits for its own pieces and lgkmcnt(0) for its own reads before
// the phase barrier, so a slot read in phase p may be restaged from phase p+1, and a piece retired in phase p may be
// read from phase p+1 (cdna_hip_programming.md §5, "Read a staged buffer one phase AFTER the wait").
//
// Persistent blocks (PERS, p.tpb > 1): the DMA of K-tiles nk, nk+1 of a slot are the next slot's K-tiles 0, 1, the
// ring state (A slot rotation, B parity) runs on across slots, so the pipeline never drains between tiles and the
// epilogue (no LDS, no barrier) runs under the next tile's first loads.  Without a next slot those pieces re-load
// this slot's last K-tile into slots never read again, so every phase issues the same loads and the waits stay static.
//
// Included by gemm_kernels.h inside namespace dllm, after the 8-phase kernel whose helpers it uses.

constexpr int PP_BN = 128;                      // tile N (tile M = 256)
constexpr int PP_AH = 16384;                    // A half-tile: 128 rows x 64 k x 2 B
constexpr int PP_BH = 8192;                     // B half-tile: 64 cols x 64 k x 2 B
constexpr int PP_LDS = 3 * PP_AH + 4 * PP_BH;   // 80 KiB: two blocks per CU

// 32-B unit swizzle of a 128-B-row MN-contiguous image: rows k and k' read by one ds_read_b64_tr_b16 lane group
// ({0,1,2,3,8,9,10,11} + 32s) land on 4 distinct units per k parity
__device__ __forceinline__ int pp_swz(int k) { return ((k >> 1) & 1) | (((k >> 3) & 1) << 1); }

template <int LAYOUT, int EPI, typename OutT, int ACT = -1, bool PERS = false>
__global__ __launch_bounds__(256, 2) void gemm_bf16_pp(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[PP_LDS];
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int ntiles = (p.M / BT_M) * (p.N / PP_BN);
  const int total = ntiles * p.ksplit;  // tile slots (split-K slices count as tiles)
  const bool pers = PERS && p.tpb > 1;
  int slot = blockIdx.x;
  auto tile_of = [&](const GemmArgs& q, int s, int& sp, int& tm0, int& tn0) {
    const int tm_ = q.M / BT_M, tn_ = q.N / PP_BN, nt = tm_ * tn_;
    const int bid0 = xcd_remap(s, nt * q.ksplit);
    sp = bid0 / nt;
    const int bid = bid0 % nt;
    const int width = q.group_m * tn_;
    const int first_m = (bid / width) * q.group_m;
    const int gsz = min(tm_ - first_m, q.group_m);
    tm0 = (first_m + (bid % width) % gsz) * BT_M;
    tn0 = ((bid % width) / gsz) * PP_BN;
  };
  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  // per-lane 32-bit byte offsets of this wave's LDS-DMA pieces: A piece q = wid + 4i (16 per half), B q = wid + 4i (8)
  uint32_t aoff[4], boff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid + 4 * i;
    if constexpr (A_KC) {  // [128 rows][64 k]: piece = 8 rows of 128 B
      const int row = 8 * q + (lane >> 3);
      aoff[i] = (uint32_t)(((long)row * p.lda + (((lane & 7) ^ ((row >> 1) & 7)) * 8)) * 2);
    } else {               // [64 k][128 mn]: piece = 4 k-rows of 256 B
      const int krow = 4 * q + (lane >> 4);
      const int u = (lane & 15) >> 1, h = lane & 1;
      aoff[i] = (uint32_t)(((long)krow * p.lda + ((u ^ mc_swz(krow)) * 16) + h * 8) * 2);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wid + 4 * i;
    if constexpr (B_KC) {  // [64 rows][64 k]
      const int row = 8 * q + (lane >> 3);
      boff[i] = (uint32_t)(((long)row * p.ldb + (((lane & 7) ^ ((row >> 1) & 7)) * 8)) * 2);
    } else {               // [64 k][64 mn]: piece = 8 k-rows of 128 B
      const int krow = 8 * q + (lane >> 3);
      const int c = lane & 7;
      boff[i] = (uint32_t)(((long)krow * p.ldb + (((c >> 1) ^ pp_swz(krow)) * 16) + (c & 1) * 8) * 2);
    }
  }
  const long a_kstep = A_KC ? BT_K : (long)BT_K * p.lda;
  const long b_kstep = B_KC ? BT_K : (long)BT_K * p.ldb;
  const long a_hstep = A_KC ? 128L * p.lda : 128L;
  const long b_hstep = B_KC ? 64L * p.ldb : 64L;
  const int nk = p.K / BT_K / p.ksplit;  // host guarantees (K/64) % ksplit == 0

  auto a_base = [&](const GemmArgs& q, int s) {
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    return (const uint16_t*)q.A + (A_KC ? (long)tm0 * q.lda : (long)tm0) + (long)sp * nk * a_kstep;
  };
  auto b_base = [&](const GemmArgs& q, int s) {
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    return (const uint16_t*)q.B + (B_KC ? (long)tn0 * q.ldb : (long)tn0) + (long)sp * nk * b_kstep;
  };
  auto slot_epilogue = [&](int s, f32x4_t (&ac)[2][2][4][2]) {
    const GemmArgs q = reload_args();
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    void* out = q.C;
    if constexpr (EPI == EPI_STORE)
      if (q.ksplit > 1) out = (char*)q.C + (long)sp * q.M * q.ldc * sizeof(OutT);
    epilogue_256<EPI, OutT, ACT, 64, 256, (ACT < 0 ? 2 : 16)>(q, ac, tm0, tn0, wr, wc, lane, out);
  };

  // K-tile bases: the current slot's panels, and the next slot's (K-tiles >= nk); without a next slot, K-tiles >= nk
  // clamp to nk - 1 (re-loads into slots never read again)
  const uint16_t* Acur = a_base(p, slot);
  const uint16_t* Bcur = b_base(p, slot);
  const uint16_t* Anext = Acur;
  const uint16_t* Bnext = Bcur;
  bool has_next = false;
  auto begin_tile = [&]() {
    const int ns = slot + (int)gridDim.x;
    has_next = pers && ns < total;
    if (has_next) {
      const GemmArgs q = reload_args();
      Anext = a_base(q, ns);
      Bnext = b_base(q, ns);
    }
  };
  begin_tile();
  // (kt - nk can reach 1 with nk == 1: clamp inside the next slot's panel too)
  auto a_kt = [&](int kt) {
    return kt < nk ? Acur + kt * a_kstep
                   : (has_next ? Anext + min(kt - nk, nk - 1) * a_kstep : Acur + (nk - 1) * a_kstep);
  };
  auto b_kt = [&](int kt) {
    return kt < nk ? Bcur + kt * b_kstep
                   : (has_next ? Bnext + min(kt - nk, nk - 1) * b_kstep : Bcur + (nk - 1) * b_kstep);
  };
  // pieces i0, i0+1 of A half hh of K-tile `src` into A slot s; piece i of B half hh into B buffer bb
  auto stage_a = [&](int i0, const uint16_t* src, int hh, int s) {
    const char* g = (const char*)(src + hh * a_hstep);
    DLLM_LDS char* dst = lds + s * PP_AH;
    glds16((const uint16_t*)(g + aoff[i0]), dst + (wid + 4 * i0) * 1024);
    glds16((const uint16_t*)(g + aoff[i0 + 1]), dst + (wid + 4 * (i0 + 1)) * 1024);
  };
  auto stage_b = [&](int i, const uint16_t* src, int hh, int bb) {
    const char* g = (const char*)(src + hh * b_hstep);
    DLLM_LDS char* dst = lds + 3 * PP_AH + (hh * 2 + bb) * PP_BH;
    glds16((const uint16_t*)(g + boff[i]), dst + (wid + 4 * i) * 1024);
  };

  // ---- per-lane fragment base addresses (LDS byte addresses, slot 0 / buffer 0) ----
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int g = lane >> 4, i15 = lane & 15;
  const int fkc = (i15 >> 1) & 7;
  const int q4 = i15 >> 2, pp = i15 & 3;
  uint32_t abase[4], bbase[2];
  if constexpr (A_KC) {
    abase[0] = lds_base + (wr * 64 + i15) * 128 + (((0 + g) ^ fkc) << 4);
    abase[1] = lds_base + (wr * 64 + i15) * 128 + (((4 + g) ^ fkc) << 4);
  } else {
    const int swz = q4 | ((g & 1) << 2);  // mc_swz(8g + q4 (+4) (+32))
#pragma unroll
    for (int t = 0; t < 4; ++t) abase[t] = lds_base + (8 * g + q4) * 256 + (((4 * wr + t) ^ swz) << 5) + 8 * pp;
  }
  const uint32_t B0 = lds_base + 3 * PP_AH;
  if constexpr (B_KC) {
    bbase[0] = B0 + (wc * 32 + i15) * 128 + (((0 + g) ^ fkc) << 4);
    bbase[1] = B0 + (wc * 32 + i15) * 128 + (((4 + g) ^ fkc) << 4);
  } else {
    const int swz2 = ((q4 >> 1) & 1) | ((g & 1) << 1);  // pp_swz(8g + q4 (+4) (+32))
#pragma unroll
    for (int t = 0; t < 2; ++t) bbase[t] = B0 + (8 * g + q4) * 128 + (((2 * wc + t) ^ swz2) << 5) + 8 * pp;
  }

  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[4][2], fb0[2][2], fb1[2][2];  // [tile][k-substep]
  s16x4_t ta_lo[4][2], ta_hi[4][2], tb_lo[2][2], tb_hi[2][2];

  // A half at LDS byte offset `so` (runtime: the ring slot) -> fa (issue only)
  auto read_a = [&](uint32_t so) {
    if constexpr (A_KC) {
      const uint32_t a0 = abase[0] + so, a1 = abase[1] + so;
      lds_b128<0 * 2048>(fa[0][0], a0); lds_b128<1 * 2048>(fa[1][0], a0);
      lds_b128<2 * 2048>(fa[2][0], a0); lds_b128<3 * 2048>(fa[3][0], a0);
      lds_b128<0 * 2048>(fa[0][1], a1); lds_b128<1 * 2048>(fa[1][1], a1);
      lds_b128<2 * 2048>(fa[2][1], a1); lds_b128<3 * 2048>(fa[3][1], a1);
    } else {
      uint32_t ab[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) ab[t] = abase[t] + so;
#define DLLM_PPA(t, s)                                   \
  lds_tr16<(s) * 8192>(ta_lo[t][s], ab[t]);              \
  lds_tr16<(s) * 8192 + 1024>(ta_hi[t][s], ab[t]);
      DLLM_PPA(0, 0) DLLM_PPA(1, 0) DLLM_PPA(2, 0) DLLM_PPA(3, 0)
      DLLM_PPA(0, 1) DLLM_PPA(1, 1) DLLM_PPA(2, 1) DLLM_PPA(3, 1)
#undef DLLM_PPA
    }
  };
  auto fin_a = [&]() {
    if constexpr (!A_KC) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) fa[t][s2] = cat_tr(ta_lo[t][s2], ta_hi[t][s2]);
    }
  };
  auto read_b = [&](uint32_t so, bf16x8_t (&fb)[2][2]) {
    if constexpr (B_KC) {
      const uint32_t b0 = bbase[0] + so, b1 = bbase[1] + so;
      lds_b128<0 * 2048>(fb[0][0], b0); lds_b128<1 * 2048>(fb[1][0], b0);
      lds_b128<0 * 2048>(fb[0][1], b1); lds_b128<1 * 2048>(fb[1][1], b1);
    } else {
      const uint32_t b0 = bbase[0] + so, b1 = bbase[1] + so;
      lds_tr16<0>(tb_lo[0][0], b0);    lds_tr16<512>(tb_hi[0][0], b0);
      lds_tr16<0>(tb_lo[1][0], b1);    lds_tr16<512>(tb_hi[1][0], b1);
      lds_tr16<4096>(tb_lo[0][1], b0); lds_tr16<4096 + 512>(tb_hi[0][1], b0);
      lds_tr16<4096>(tb_lo[1][1], b1); lds_tr16<4096 + 512>(tb_hi[1][1], b1);
    }
  };
  auto fin_b = [&](bf16x8_t (&fb)[2][2]) {
    if constexpr (!B_KC) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) fb[t][s2] = cat_tr(tb_lo[t][s2], tb_hi[t][s2]);
    }
  };
  auto mfma_quad = [&](f32x4_t (&c)[4][2], const bf16x8_t (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          c[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt][s2], fa[mt][s2], c[mt][nt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // optional skew: the odd workgroup slot of the CU (HW_ID.TG_ID) starts later, so the two co-resident blocks do
  // not run their read / barrier / MFMA segments in lockstep
  if (p.skew > 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));  // hwreg(HW_REG_HW_ID)
    if ((hw >> 16) & 1)
      for (int i = 0; i < p.skew; ++i) __builtin_amdgcn_s_sleep(1);
  }
  // ring state (runs on across persistent slots): A slots of A-h0 / A-h1 of the current K-tile, B buffer parity
  int sa0 = 0, sa1 = 1, bb = 0;
  // prologue = the loads phases q1(-2) .. q3(-1) would have issued, in that order: A0(0) B0(0) B1(0) | A1(0) B0(1)
  // A0(1)[0,1] B1(1)[0]; vmcnt(9) leaves the last 9 in flight (they are retired by the loop's own waits)
  {
    const uint16_t* A0 = a_kt(0);
    const uint16_t* B0p = b_kt(0);
    const uint16_t* A1 = a_kt(1);
    const uint16_t* B1p = b_kt(1);
    stage_a(0, A0, 0, 0); stage_a(2, A0, 0, 0);
    stage_b(0, B0p, 0, 0); stage_b(1, B0p, 0, 0);
    stage_b(0, B0p, 1, 0); stage_b(1, B0p, 1, 0);
    stage_a(0, A0, 1, 1); stage_a(2, A0, 1, 1);
    stage_b(0, B1p, 0, 1); stage_b(1, B1p, 0, 1);
    stage_a(0, A1, 0, 2);
    stage_b(0, B1p, 1, 1);
  }
  asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  DLLM_BARRIER();

#define DLLM_PP_END(W)                                       \
  if (W) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");    \
  DLLM_LDS_WAIT();                                           \
  DLLM_BARRIER();

  for (;;) {  // slots of this block (one pass unless persistent)
    for (int kk = 0; kk < nk; ++kk) {
      const int s3 = 3 - sa0 - sa1;  // slot of A-h0(kk+1)
      const uint16_t* A1p = a_kt(kk + 1);
      const uint16_t* A2p = a_kt(kk + 2);
      const uint16_t* B1p = b_kt(kk + 1);
      const uint16_t* B2p = b_kt(kk + 2);
      const uint32_t bo = (uint32_t)bb * PP_BH;  // B buffer of K-tile kk (halves at +0 / +2 * PP_BH)
      // q0: quadrant (0,0)
      read_a((uint32_t)sa0 * PP_AH); read_b(bo, fb0);
      stage_b(1, B1p, 1, bb ^ 1);
      stage_a(2, A1p, 0, s3);
      DLLM_PP_END(false)
      fin_a(); fin_b(fb0);
      mfma_quad(acc[0][0], fb0);
      // q1: quadrant (0,1)
      read_b(bo + 2 * PP_BH, fb1);
      stage_a(0, A1p, 1, sa0);
      stage_b(0, B2p, 0, bb);
      DLLM_PP_END(true)
      fin_b(fb1);
      mfma_quad(acc[0][1], fb1);
      // q2: quadrant (1,1)
      read_a((uint32_t)sa1 * PP_AH);
      stage_a(2, A1p, 1, sa0);
      stage_b(1, B2p, 0, bb);
      DLLM_PP_END(false)
      fin_a();
      mfma_quad(acc[1][1], fb1);
      // q3: quadrant (1,0)
      stage_a(0, A2p, 0, sa1);
      stage_b(0, B2p, 1, bb);
      DLLM_PP_END(true)
      mfma_quad(acc[1][0], fb0);
      // rotate: A-h0(kk+1) in s3, A-h1(kk+1) in sa0
      sa1 = sa0;
      sa0 = s3;
      bb ^= 1;
    }
    if (!has_next) break;
    // Persistent: the next slot's K-tiles 0/1 are landed or in flight; this slot's epilogue runs meanwhile (no LDS,
    // no barrier: the barrier sequence continues into the next slot's q0; its memory operations are older than the
    // next slot's loads and are retired by its counted waits)
    slot_epilogue(slot, acc);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    slot += (int)gridDim.x;
    Acur = Anext;
    Bcur = Bnext;
    begin_tile();
  }
#undef DLLM_PP_END
  // drain the tail prefetches before the block can release its LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  slot_epilogue(slot, acc);
}

