// High-throughput bf16 "NT" GEMM for the wide-MLP path (gfx950):
//
//   C[M][N] = A[M][K] . B[N][K]^T      (both operands k-contiguous, bf16; fp32 accumulate)
//
// The wide client (fedmi/fl/wide.py) keeps every operand k-contiguous -- activations and
// deltas are also written transposed by the epilogues, and W^T is re-quantised after each
// optimizer step -- so forward (X W^T), dgrad (dY W) and wgrad (dY^T X) are all this
// kernel.  Structure (CDNA guide §5, "standard MFMA GEMM main loop"):
//   * 128x128 block tile, BK = 64, 256 threads = 4 waves in 2x2, 64x64 per wave
//     (4x4 tiles of v_mfma_f32_16x16x32_bf16, 64 fp32 accumulators per lane);
//   * operands staged global -> LDS by 16-byte LDS-DMA (global_load_lds_dwordx4: no VGPR
//     round trip); double-buffered variant issues tile k+1's DMA before tile k's MFMAs;
//   * LDS rows of 128 B with the 16-byte chunk index XOR-swizzled by (row >> 1) & 7, so the
//     16 rows read by one ds_read_b128 lane group land on 16 distinct bank slots (T2);
//   * XCD-aware block remap (T1); fused epilogue: alpha, +bias, ReLU, +beta*C, fp32 and/or
//     bf16 row-major and bf16 transposed outputs.
// Requires M % 128 == N % 128 == K % 64 == 0 (the host falls back to gemm_mfma.hip).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <cstdlib>

#include "gemm_nt_bf16.h"
#include "gemm_mfma.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define NT_BM 128
#define NT_BN 128
#define NT_BK 64
#define NT_THREADS 256

// byte offset of 16-byte chunk c (0..7) of row r in a [128][64] bf16 LDS tile
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ int xcd_remap_nt(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One 16-byte global -> LDS DMA per lane (global_load_lds_dwordx4).  The LDS destination is
// wave-uniform base + lane * 16, so the swizzle lives in the per-lane GLOBAL address.
__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_base, 16, 0, 0);
}

// The same DMA through a buffer resource (buffer_load_dwordx4 ... lds, the form hipBLASLt's
// MT256x256x64 kernels use): base in SGPRs, a lane VGPR offset shared by every piece of the same
// swizzle parity, the piece / K-tile offset in an SGPR (soffset).  Bounds: the whole 32-bit range
// from the block's base (the operands' extents are checked on the host).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nt_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* lds_base) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_base, 16, voff, soff, 0, 0);
}

// DB = 0: one LDS buffer (32 KiB), two barriers per K-step, ~3 blocks/CU hide the DMA.
// DB = 1: two LDS buffers (64 KiB), the DMA of tile k+1 overlaps the MFMAs of tile k.
template <int DB>
__global__ void __launch_bounds__(NT_THREADS)
gemm_nt_bf16_kernel(NTArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[(DB + 1) * 2 * NT_BM * NT_BK * 2];
    constexpr int TILE = NT_BM * NT_BK * 2;  // bytes per operand tile
    const int mt = g.M / NT_BM, nt = g.N / NT_BN;
    const int bid = xcd_remap_nt(blockIdx.x, mt * nt);
    const int m0 = (bid % mt) * NT_BM, n0 = (bid / mt) * NT_BN;
    const __hip_bfloat16* A = reinterpret_cast<const __hip_bfloat16*>(g.A);
    const __hip_bfloat16* B = reinterpret_cast<const __hip_bfloat16*>(g.B);
    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    const int lr = lane & 15, lg = lane >> 4;

    // DMA map: wave w issues 1-KiB pieces q = 4w + i (rows 8q .. 8q+7) of each operand;
    // lane l lands at LDS row 8q + l/8, physical chunk l%8 = logical chunk (l%8) ^ f(row).
    const __hip_bfloat16* srcA[4];
    const __hip_bfloat16* srcB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 8 * (4 * wave + i) + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        srcA[i] = A + (size_t)(m0 + row) * g.lda + c * 8;
        srcB[i] = B + (size_t)(n0 + row) * g.ldb + c * 8;
    }
    auto dma = [&](int k0, int buf) {
        char* base = smem + buf * 2 * TILE;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            glds16(srcA[i] + k0, base + (4 * wave + i) * 1024);
            glds16(srcB[i] + k0, base + TILE + (4 * wave + i) * 1024);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const char* As = smem + buf * 2 * TILE;
        const char* Bs = As + TILE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // two 32-deep MFMA k-steps per 64-deep tile
            bf16x8 af[4], bf[4];
            const int chunk = ks * 4 + lg;  // lane group lg holds k = 8*lg .. 8*lg+7 of the step
#pragma unroll
            for (int x = 0; x < 4; ++x) af[x] = *reinterpret_cast<const bf16x8*>(As + swz(wm + 16 * x + lr, chunk));
#pragma unroll
            for (int y = 0; y < 4; ++y) bf[y] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn + 16 * y + lr, chunk));
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[x], bf[y], acc[x][y], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
    };

    const int ktiles = g.K / NT_BK;
    if (DB) {
        dma(0, 0);
        for (int kt = 0; kt < ktiles; ++kt) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // tile kt visible to all waves; buffer (kt+1)&1 no longer read
            if (kt + 1 < ktiles) dma((kt + 1) * NT_BK, (kt + 1) & 1);
            compute(kt & 1);
        }
    } else {
        for (int kt = 0; kt < ktiles; ++kt) {
            dma(kt * NT_BK, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            compute(0);
            __syncthreads();
        }
    }

    // epilogue (C/D map: col = lane&15, row = 4*(lane>>4) + j)
    __hip_bfloat16* Cb = reinterpret_cast<__hip_bfloat16*>(g.Cbf16);
    __hip_bfloat16* CbT = reinterpret_cast<__hip_bfloat16*>(g.CbT);
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        const int n = n0 + wn + 16 * y + lr;
        const float bv = g.bias != nullptr ? g.bias[n] : 0.f;
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int mm = m0 + wm + 16 * x + 4 * lg + j;
                float v = acc[x][y][j] * g.alpha + bv;
                if (g.relu) v = fmaxf(v, 0.f);
                if (g.mask != nullptr) {
                    const __hip_bfloat16 mk = reinterpret_cast<const __hip_bfloat16*>(g.mask)[(size_t)mm * g.ldmask + n];
                    v = __bfloat162float(mk) > 0.f ? v : 0.f;
                }
                if (g.C != nullptr) {
                    float* cp = g.C + (size_t)mm * g.ldc + n;
                    if (g.beta != 0.f) v += g.beta * *cp;
                    *cp = v;
                }
                if (Cb != nullptr) Cb[(size_t)mm * g.ldcb + n] = __float2bfloat16(v);
                if (CbT != nullptr) CbT[(size_t)n * g.ldct + mm] = __float2bfloat16(v);
            }
    }
}

// ---------------------------------------------------------------------------------------------
// 256x256 ping-pong variant (variant 2; M % 256 == N % 256 == 0, K % 64 == 0).
//
// 512 threads = 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave (8x4 16x16 tiles, 128 fp32
// accumulators per lane).  A K-tile (BK = 64) is computed in four PHASES of 16 MFMAs each:
//     r = 0: rows m0 (first 64 of the wave's 128) x k 0..31     r = 1: rows m1 x k 0..31
//     r = 2: rows m1 x k 32..63                                r = 3: rows m0 x k 32..63
// LDS holds two K-tiles (2 x 64 KiB, one __shared__ array), each as k-halves [ks][256][32] of
// 64-byte rows with the 16-byte chunk index XOR-ed with (row >> 2) & 2: a ds_read_b128 is
// serviced in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32), and with this
// swizzle each group's 16 (row, chunk) pairs hit 16 distinct 16-byte bank slots (a plain
// (row >> 2) & 3 XOR leaves them 2-way conflicted).  A K-tile is 8 LDS-DMAs per lane (8 KiB
// per block each), numbered in first-read order: d0 A m0 ks0 | d1,d2 B ks0 | d3 A m1 ks0 |
// d4 A m1 ks1 | d5,d6 B ks1 | d7 A m0 ks1  (first read in phases 0,0,0,1,2,2,2,3).
//
// Schedule, global phase g = 4 * tile + r, each wave:
//     MEM(g):  2 LDS-DMAs (r = 0: tile+1 d4,d5 | 1: tile+1 d6,d7 | 2: tile+2 d0,d1 |
//              3: tile+2 d2,d3 -- every slot restaged >= 2 phases after its last read, and
//              4-6 phases before its first), ds_read phase g's fragments, then
//              s_waitcnt vmcnt(N) retiring every DMA first read in phase g + 1
//              (N = DMAs still needed later: 10 for even r, 9 for odd r)
//     s_barrier; s_waitcnt lgkmcnt(0); 16 MFMAs; s_barrier
// The second wave row starts one barrier later, so on every SIMD one wave's MFMA cluster runs
// while the other wave's MEM section (DMA issue, LDS reads, vmcnt wait) runs.  A DMA's data is
// read at least one barrier after every wave's vmcnt that retires it (group 0: the barrier
// after the wait; group 1: one barrier later still); a slot is restaged two phases after its
// last read, i.e. after a barrier that follows every reader's lgkmcnt(0).  The last two
// K-tiles issue nothing past the end and drain with vmcnt(0).
#define NT2_BM 256
#define NT2_THREADS 512

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Epilogue of the 256x256 loops (ping-pong and full-line): the block's 256x256 bf16 output tile is
// staged through the (now free) 128 KiB of LDS; see the comment inside.
// Output configuration of an epilogue as compile-time flags (NT_EPI_*), so the unrolled
// 128-element epilogue carries no per-element runtime branches or dead paths; -1 = read the
// configuration from the arguments at run time.
#define NT_EPI_C 1
#define NT_EPI_CB 2
#define NT_EPI_CBT 4
#define NT_EPI_MASK 8
#define NT_EPI_RELU 16
#define NT_EPI_BIAS 32
#define NT_EPI_BETA 64
#define NT_EPI_CSUM 128
static inline int nt_epi_flags(const NTArgs& g) {
    return (g.C != nullptr ? NT_EPI_C : 0) | (g.Cbf16 != nullptr ? NT_EPI_CB : 0) | (g.CbT != nullptr ? NT_EPI_CBT : 0) |
           (g.mask != nullptr ? NT_EPI_MASK : 0) | (g.relu ? NT_EPI_RELU : 0) | (g.bias != nullptr ? NT_EPI_BIAS : 0) |
           (g.C != nullptr && g.beta != 0.f ? NT_EPI_BETA : 0) | (g.csum != nullptr ? NT_EPI_CSUM : 0);
}

// NW = 8 waves as 2 x 4 (128 x 64 outputs per wave, acc[8][4]; variants 2 / 3) or NW = 4 waves as
// 2 x 2 (128 x 128, acc[8][8]: the four-wave loops measured in rounds 3 and 5,
// profiles/nt_four_wave_r3_rejected.log, profiles/nt_ring_bufdma_r5.log).
template <int F, int NW = 8>
__device__ __forceinline__ void pp_epilogue(const NTArgs& g, char* smem, f32x4 (&acc)[8][32 / NW], int m0, int n0,
                                            int w, int l) {
    constexpr int YT = 32 / NW, WN = 16 * YT;  // 16-column tiles per wave, columns per wave
    constexpr int RI = 256 / (2 * NW);          // row-pair iterations of the block-wide loops
    const int wr = w / (NW / 2), wc = w % (NW / 2);
    const int lr = l & 15, lg = l >> 4;
    const bool hC = F < 0 ? g.C != nullptr : (F & NT_EPI_C) != 0;
    const bool hCb = F < 0 ? g.Cbf16 != nullptr : (F & NT_EPI_CB) != 0;
    const bool hCbT = F < 0 ? g.CbT != nullptr : (F & NT_EPI_CBT) != 0;
    const bool hMask = F < 0 ? g.mask != nullptr : (F & NT_EPI_MASK) != 0;
    const bool hRelu = F < 0 ? g.relu != 0 : (F & NT_EPI_RELU) != 0;
    const bool hBias = F < 0 ? g.bias != nullptr : (F & NT_EPI_BIAS) != 0;
    const bool hBeta = F < 0 ? g.beta != 0.f : (F & NT_EPI_BETA) != 0;
    const bool hCsum = F < 0 ? g.csum != nullptr : (F & NT_EPI_CSUM) != 0;

    // Epilogue.  Every wave's LDS reads retired before that last barrier, so the 128 KiB of LDS
    // now holds the block's 256x256 bf16 output tile as 512-byte rows whose 16-byte chunk index
    // is XOR-ed with sw(row) = ((row >> 2) & 3) * 2 (the four 4-row lane groups of a 2-byte
    // write land on distinct banks; a 16-lane read of 16 chunks of one row stays conflict-free).
    // Each lane drops its bf16 values into the tile, then the block stores it with full 512-byte
    // row segments (16 B per lane) instead of 2-byte scattered stores.  The dgrad ReLU mask is
    // DMA-ed into the same slots first (full-line loads, same swizzle) and overwritten in place
    // by the lane that reads it.
    auto sw = [](int row) { return ((row >> 2) & 3) * 2; };
    auto tile_off = [&](int row, int col) { return row * 512 + ((((col >> 3) ^ sw(row))) << 4) + (col & 7) * 2; };
    __hip_bfloat16* Cb = reinterpret_cast<__hip_bfloat16*>(g.Cbf16);
    __hip_bfloat16* CbT = reinterpret_cast<__hip_bfloat16*>(g.CbT);
    if (hMask) {
        const __hip_bfloat16* Mk = reinterpret_cast<const __hip_bfloat16*>(g.mask);
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const int row = i * 2 * NW + w * 2, rr = row + (l >> 5);
            glds16(Mk + (size_t)(m0 + rr) * g.ldmask + n0 + (((l & 31) ^ sw(rr)) << 3), smem + row * 512);
        }
        vm_wait<0>();
        __syncthreads();
    }

#pragma unroll
    for (int y = 0; y < YT; ++y) {
        const int cl = wc * WN + 16 * y + lr, n = n0 + cl;
        const float bv = hBias ? g.bias[n] : 0.f;
        float cs = 0.f;  // column n's sum over the lane's 32 rows of the bf16 output (hCsum)
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            uint32_t tp[2];  // the lane's 4 consecutive rows of column n, packed for CbT
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int rl = wr * 128 + 16 * x + 4 * lg + j, mm = m0 + rl;
                __hip_bfloat16* slot = reinterpret_cast<__hip_bfloat16*>(smem + tile_off(rl, cl));
                float v = acc[x][y][j] * g.alpha + bv;
                if (hRelu) v = fmaxf(v, 0.f);
                if (hMask) v = __bfloat162float(*slot) > 0.f ? v : 0.f;
                if (hC) {
                    float* cp = g.C + (size_t)mm * g.ldc + n;
                    if (hBeta) v += g.beta * *cp;
                    *cp = v;
                }
                const __hip_bfloat16 hv = __float2bfloat16(v);
                if (hCb) *slot = hv;
                if (hCsum) cs += __bfloat162float(hv);
                const uint32_t hb = __bfloat16_as_ushort(hv);
                if (j & 1) tp[j >> 1] |= hb << 16;
                else tp[j >> 1] = hb;
            }
            if (hCbT) {  // 8-byte store: rows mm .. mm+3 are contiguous in CbT's row n
                const size_t off = (size_t)n * g.ldct + m0 + wr * 128 + 16 * x + 4 * lg;
                *reinterpret_cast<uint2*>(CbT + off) = make_uint2(tp[0], tp[1]);
            }
        }
        if (hCsum) {
            // + the other three lane groups of the column (fixed order): the wave's 128 rows
            cs += __shfl_xor(cs, 16);
            cs += __shfl_xor(cs, 32);
            if (lg == 0) g.csum[(size_t)((m0 >> 7) + wr) * g.ldcs + n] = cs;
        }
    }
    if (hCb) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const int rr = i * 2 * NW + w * 2 + (l >> 5), p = l & 31;
            const uint4 d = *reinterpret_cast<const uint4*>(smem + rr * 512 + p * 16);
            *reinterpret_cast<uint4*>(Cb + (size_t)(m0 + rr) * g.ldcb + n0 + ((p ^ sw(rr)) << 3)) = d;
        }
    }
}

__global__ void __launch_bounds__(NT2_THREADS)
gemm_nt_bf16_pp_kernel(NTArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 65536];
    const int mt = g.M / NT2_BM, nt = g.N / NT2_BM;
    const int bid = xcd_remap_nt(blockIdx.x, mt * nt);
    // grouped tile order: the ~32 blocks an XCD runs at once (consecutive bids after the XCD
    // remap) cover 8 m-tiles x 4 n-tiles, so each K-slice of A and B is fetched into that XCD's
    // L2 once per 12 panels instead of once per 33 (m-major order)
    constexpr int GM = 8;
    const int grp = bid / (GM * nt), first_m = grp * GM;
    const int gsz = min(mt - first_m, GM);
    const int in_grp = bid - grp * GM * nt;
    const int m0 = (first_m + in_grp % gsz) * NT2_BM, n0 = (in_grp / gsz) * NT2_BM;
    const __hip_bfloat16* A = reinterpret_cast<const __hip_bfloat16*>(g.A);
    const __hip_bfloat16* B = reinterpret_cast<const __hip_bfloat16*>(g.B);
    const int t = threadIdx.x;
    // wave index in an SGPR: LDS-DMA destinations (M0) and row bases become scalar, each DMA is
    // one global_load_lds with an SGPR base + 32-bit lane offset (no 64-bit VALU address adds;
    // measured 1.5-4 % faster than per-lane 64-bit source pointers)
    const int w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
    const int wr = w >> 2, wc = w & 3;
    const int lr = l & 15, lg = l >> 4;

    // DMA sources: lane l of wave w fills LDS row (16-row group base) + l/4, physical chunk l%4
    // = logical chunk (l%4) ^ (((row>>2)&3) & 2) of the row's 64-byte k-half.
    const int dchunk = ((l & 3) ^ ((l >> 4) & 2)) * 8;
    int dstA[2], dstB[2];
    const char* sbA[2];
    const char* sbB[2];
    const uint32_t voA = (uint32_t)(((l >> 2) * g.lda + dchunk) * 2);
    const uint32_t voB = (uint32_t)(((l >> 2) * g.ldb + dchunk) * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ra = (w >> 2) * 128 + h * 64 + (w & 3) * 16;  // A piece m-half h
        sbA[h] = reinterpret_cast<const char*>(A + (size_t)(m0 + ra) * g.lda);
        dstA[h] = ra * 64;
        const int rb = h * 128 + w * 16;                         // B piece, DMA h of 2
        sbB[h] = reinterpret_cast<const char*>(B + (size_t)(n0 + rb) * g.ldb);
        dstB[h] = 32768 + rb * 64;
    }
    // LDS-DMA d (0..7) of K-tile `tile`, in first-read order: d0 A m0 ks0, d1-d2 B ks0, d3 A m1
    // ks0, d4 A m1 ks1, d5-d6 B ks1, d7 A m0 ks1 (first read in phases 0,0,0,1,2,2,2,3)
    auto dma = [&](int tile, int d) {
        const int ks = (d >= 4) ? 1 : 0;
        const int kb = (tile * 64 + ks * 32) * 2;
        char* base = smem + (tile & 1) * 65536 + ks * 16384;
        if (d == 0 || d == 7) glds16(sbA[0] + kb + voA, base + dstA[0]);
        else if (d == 3 || d == 4) glds16(sbA[1] + kb + voA, base + dstA[1]);
        else if (d == 1 || d == 5) glds16(sbB[0] + kb + voB, base + dstB[0]);
        else glds16(sbB[1] + kb + voB, base + dstB[1]);
    };

    // fragment read offset of this lane inside a 16-row group: row lr, chunk lg swizzled
    const int foff = lr * 64 + ((lg ^ ((lr >> 2) & 2)) << 4);
    const int aoff = wr * 128 * 64 + foff, boff = 32768 + wc * 64 * 64 + foff;

    f32x4 acc[8][4];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
    bf16x8 af[4], bfr[4];

    const int KT = g.K / 64;
    // prologue: what phases -6 .. -1 would have issued (tile 0, then tile 1's d0-d3); retire
    // phase 0's DMAs (tile 0 d0-d2), leaving 5 + 4 = 9 in flight
    dma(0, 0); dma(0, 1); dma(0, 2); dma(0, 3); dma(0, 4); dma(0, 5); dma(0, 6); dma(0, 7);
    if (KT > 1) { dma(1, 0); dma(1, 1); dma(1, 2); dma(1, 3); }
    if (KT > 2) vm_wait<9>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();

    // two DMAs per phase, issued before the fragment reads: r = 0: tile+1 d4,d5; r = 1: tile+1
    // d6,d7; r = 2: tile+2 d0,d1; r = 3: tile+2 d2,d3 (each slot restaged >= 2 phases after its
    // last read).  (Measured alternatives: after the fragment reads or inside the MFMA cluster,
    // 1-6 % slower; profiles/nt_ksweep_r1_experiments.log.)
    auto phase = [&](int q, int r, bool tail) {
        const char* buf = smem + ((q >> 2) & 1) * 65536 + ((r >= 2) ? 16384 : 0);
        const int mh = (r == 1 || r == 2) ? 1 : 0;
        const int dtile = (q >> 2) + (r < 2 ? 1 : 2);
        const int dd = (r < 2) ? 4 + 2 * r : 2 * (r - 2);
        if (!tail || dtile < KT) {
            dma(dtile, dd);
            dma(dtile, dd + 1);
        }
        if ((r & 1) == 0) {
#pragma unroll
            for (int y = 0; y < 4; ++y) bfr[y] = *reinterpret_cast<const bf16x8*>(buf + boff + y * 16 * 64);
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
            af[x] = *reinterpret_cast<const bf16x8*>(buf + aoff + (mh * 64 + x * 16) * 64);
        if (tail) vm_wait<0>();
        else if ((r & 1) == 0) vm_wait<10>();
        else vm_wait<9>();
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
                acc[mh * 4 + x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[x], bfr[y], acc[mh * 4 + x][y], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
    };

    int kt = 0;
    for (; kt + 2 < KT; ++kt) {
        phase(4 * kt + 0, 0, false);
        phase(4 * kt + 1, 1, false);
        phase(4 * kt + 2, 2, false);
        phase(4 * kt + 3, 3, false);
    }
    for (; kt < KT; ++kt) {
        phase(4 * kt + 0, 0, true);
        phase(4 * kt + 1, 1, true);
        phase(4 * kt + 2, 2, true);
        phase(4 * kt + 3, 3, true);
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // match the second wave row's extra barrier
    pp_epilogue<-1>(g, smem, acc, m0, n0, w, l);
}

// ---------------------------------------------------------------------------------------------
// 256x256 full-line variant (variant 3): variant 2's ping-pong phase structure (8 waves as 2 x 4,
// four phases of 16 MFMAs per K-tile, counted vmcnt + raw barriers, staggered wave rows, same
// per-element k order -- bit-identical results), with the operand tiles held as 128-byte LDS
// rows (both k-halves of a row) and every LDS-DMA a piece of 8 WHOLE 128-byte lines (variant 2:
// 16 half lines).  The timing experiment that moved variant 2's DMAs onto whole lines ran the
// main loop 6-10 % faster (profiles/nt_ksweep_r1_experiments.log).
//
// LDS: two K-tile buffers of 64 KiB (tile parity), A [256][128 B] then B [256][128 B]; 16-byte
// chunk c of row r at chunk c ^ ((r >> 1) & 7), which keeps every ds_read_b128 lane group on
// 16 distinct bank slots.  A DMA piece is rows 8q .. 8q+7 of one operand: lane l lands at row
// 8q + l/8, physical chunk l%8 (LDS-linear), fetched from logical chunk (l%8) ^ ((row >> 1) & 7).
//
// A piece can only be restaged >= 2 phases after the LAST phase that reads either k-half of its
// rows (a phase's reads retire at the lgkmcnt(0) after its first barrier, and the other wave row
// runs one barrier behind).  Phases read: r = 0: B ks0 + A m0 ks0 | r = 1: A m1 ks0 + B ks1
// (fetched a phase early, so B's rows are done after phase 1) | r = 2: A m1 ks1 | r = 3: A m0 ks1.
// DMA schedule for K-tile u (2 pieces per wave per phase, 8 per K-tile):
//     phase (u-2).3: B pieces 0,1 | (u-1).0: B pieces 2,3 | (u-1).1: A m0 | (u-1).2: A m1
// -- 2-4 phases after the last read of the slot's previous tile, 3-5 phases ahead of the first
// read.  Waits (before a phase's first barrier, retiring what the NEXT phase reads; pieces still
// allowed in flight, in issue order): r = 0: 4 (B01, B23 of u+1) | r = 3: 4 (A m1 of u+1, B01 of
// u+2) | r = 1, 2: none.
#ifndef NT_MFMA_YX
#define NT_MFMA_YX 0
#endif
#ifndef NT_PRIO
#define NT_PRIO 1   // issue priority of a phase's MFMA cluster (A/B builds)
#endif
template <int F, bool BUF = false>
__global__ void __launch_bounds__(NT2_THREADS)
gemm_nt_bf16_fl_kernel(NTArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 65536];
#define NT_STAMP(i)                                                                              \
    if (g.dbg != nullptr && threadIdx.x == 0) g.dbg[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime()
    NT_STAMP(0);
    const int mt = g.M / NT2_BM, nt = g.N / NT2_BM;
#ifdef NT_PERSIST
    // (A/B) one resident block per CU walks tiles blockIdx.x, + gridDim.x, ...: the next tile's
    // prologue DMAs start while the previous tile's output stores drain (gridDim.x % 8 == 0, so a
    // virtual block keeps the XCD of the block that runs it and the remap below is unchanged)
    for (int vb = blockIdx.x; vb < mt * nt; vb += gridDim.x) {
#else
    {
        const int vb = blockIdx.x;
#endif
    const int bid = xcd_remap_nt(vb, mt * nt);
#ifndef NT_GM
#define NT_GM 4
#endif
    constexpr int GM = NT_GM;  // grouped tile order: 4 m-tiles per group (8: -3.5 % at 16384x4096x8192, profiles/nt_gm_r6.log)
    const int grp = bid / (GM * nt), first_m = grp * GM;
    const int gsz = min(mt - first_m, GM);
    const int in_grp = bid - grp * GM * nt;
    const int m0 = (first_m + in_grp % gsz) * NT2_BM, n0 = (in_grp / gsz) * NT2_BM;
    const __hip_bfloat16* A = reinterpret_cast<const __hip_bfloat16*>(g.A);
    const __hip_bfloat16* B = reinterpret_cast<const __hip_bfloat16*>(g.B);
    const int t = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
    const int wr = w >> 2, wc = w & 3;
    const int lr = l & 15, lg = l >> 4;

    // lane offsets of a piece (bytes from the piece's first source row): row 8q + l/8, logical
    // chunk (l%8) ^ ((4q + l/16) & 7) -- depends on the parity of q only
    uint32_t voA[2], voB[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int c = (l & 7) ^ ((4 * par + (l >> 4)) & 7);
        voA[par] = (uint32_t)(((l >> 3) * g.lda + c * 8) * 2);
        voB[par] = (uint32_t)(((l >> 3) * g.ldb + c * 8) * 2);
    }
    // this wave's pieces: B rows 32w + 8i (i = 0..3); A m0 rows rm0 + 8i, A m1 rows rm0 + 64 + 8i
    // (i = 0, 1) with rm0 = 16w (w < 4) or 128 + 16(w - 4): piece parities are i & 1
    const int rm0 = (w < 4) ? 16 * w : 128 + 16 * (w - 4);
    const char* sbB = reinterpret_cast<const char*>(B + (size_t)(n0 + 32 * w) * g.ldb);
    const char* sbA0 = reinterpret_cast<const char*>(A + (size_t)(m0 + rm0) * g.lda);
    const char* sbA1 = reinterpret_cast<const char*>(A + (size_t)(m0 + rm0 + 64) * g.lda);
    const size_t rowB8 = (size_t)8 * g.ldb * 2, rowA8 = (size_t)8 * g.lda * 2;
    // BUF (the default; variant 10 = without): the pieces through buffer resources (blds16), offsets in SGPRs
    const __amdgpu_buffer_rsrc_t rsB = nt_rsrc(sbB), rsA = nt_rsrc(sbA0);
    const uint32_t rowA64 = (uint32_t)((size_t)64 * g.lda * 2);  // < 2^31: checked in gemm_nt_bf16_launch
    auto dmaB = [&](int tile, int i) {
        char* dst = smem + (tile & 1) * 65536 + 32768 + (32 * w + 8 * i) * 128;
        if (BUF) blds16(rsB, voB[i & 1], (uint32_t)(i * rowB8) + tile * 128, dst);
        else glds16(sbB + i * rowB8 + tile * 128 + voB[i & 1], dst);
    };
    auto dmaA = [&](int tile, int half, int i) {
        char* dst = smem + (tile & 1) * 65536 + (rm0 + 64 * half + 8 * i) * 128;
        if (BUF) {
            blds16(rsA, voA[i & 1], half * rowA64 + (uint32_t)(i * rowA8) + tile * 128, dst);
        } else {
            const char* src = (half ? sbA1 : sbA0) + i * rowA8 + tile * 128 + voA[i & 1];
            glds16(src, dst);
        }
    };

    // fragment reads: row (16-row group base) + lr, chunk 4 ks + lg swizzled by (lr >> 1) & 7
    const int f = (lr >> 1) & 7;
    const int fo0 = lr * 128 + ((lg ^ f) << 4), fo1 = lr * 128 + (((4 + lg) ^ f) << 4);
    const int aoff = wr * 128 * 128, boff = 32768 + wc * 64 * 128;

    f32x4 acc[8][4];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
    bf16x8 af[4], bfr[4], bfr1[4];

    const int KT = g.K / 64;
    // prologue: what phases (-2).3 .. (-1).3 would have issued -- tile 0, then tile 1's B01
    dmaB(0, 0); dmaB(0, 1); dmaB(0, 2); dmaB(0, 3);
    dmaA(0, 0, 0); dmaA(0, 0, 1); dmaA(0, 1, 0); dmaA(0, 1, 1);
    if (KT > 1) {
        dmaB(1, 0); dmaB(1, 1);
        vm_wait<4>();  // phase 0 reads B and A m0 of tile 0
    } else {
        vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
#ifndef NT_NO_STAGGER
    if (wr == 1) __builtin_amdgcn_s_barrier();   // the second wave row runs one barrier behind
#endif
    NT_STAMP(1);

    auto phase = [&](int kt, int r, bool tail) {
        const char* buf = smem + (kt & 1) * 65536;
        const int mh = (r == 1 || r == 2) ? 1 : 0;
        const int fo = (r >= 2) ? fo1 : fo0;
        auto issue = [&]() {
            if (r == 0) {
                if (!tail || kt + 1 < KT) { dmaB(kt + 1, 2); dmaB(kt + 1, 3); }
            } else if (r == 1) {
                if (!tail || kt + 1 < KT) { dmaA(kt + 1, 0, 0); dmaA(kt + 1, 0, 1); }
            } else if (r == 2) {
                if (!tail || kt + 1 < KT) { dmaA(kt + 1, 1, 0); dmaA(kt + 1, 1, 1); }
            } else {
                if (!tail || kt + 2 < KT) { dmaB(kt + 2, 0); dmaB(kt + 2, 1); }
            }
        };
#ifdef NT_DMA_FIRST
        issue();   // (A/B: the round-5 order, DMA issue ahead of the phase's fragment reads)
#endif
        if (r == 0) {
#pragma unroll
            for (int y = 0; y < 4; ++y) bfr[y] = *reinterpret_cast<const bf16x8*>(buf + boff + y * 16 * 128 + fo0);
        } else if (r == 1) {
#pragma unroll
            for (int y = 0; y < 4; ++y) bfr1[y] = *reinterpret_cast<const bf16x8*>(buf + boff + y * 16 * 128 + fo1);
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
            af[x] = *reinterpret_cast<const bf16x8*>(buf + aoff + (mh * 64 + x * 16) * 128 + fo);
#ifndef NT_DMA_FIRST
        issue();   // after the fragment reads: 0.5-1 % faster at the wide shapes (profiles/nt_gm_r6.log)
#endif
        // the last two K-tiles issue fewer pieces: exact counts there too (a vmcnt(0) right after
        // an issue would expose a whole DMA latency per phase)
        if (!tail || kt + 2 < KT) {
            if (r == 0 || r == 3) vm_wait<4>();
        } else if (kt + 2 == KT) {
            if (r == 0) vm_wait<4>();       // A m1 of kt; B01, B23 of kt+1 may fly
            else if (r == 3) vm_wait<2>();  // B, A m0 of kt+1; its A m1 may fly
        } else if (r == 0) {
            vm_wait<0>();                   // last tile: its A m1
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (NT_PRIO > 0) __builtin_amdgcn_s_setprio(NT_PRIO);
        // (NT_MFMA_YX: B-fragment-major issue order, A/B; independent accumulators either way)
        if (r <= 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int x = NT_MFMA_YX ? (i & 3) : (i >> 2), y = NT_MFMA_YX ? (i >> 2) : (i & 3);
                acc[mh * 4 + x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[x], bfr[y], acc[mh * 4 + x][y], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int x = NT_MFMA_YX ? (i & 3) : (i >> 2), y = NT_MFMA_YX ? (i >> 2) : (i & 3);
                acc[mh * 4 + x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[x], bfr1[y], acc[mh * 4 + x][y], 0, 0, 0);
            }
        }
        if (NT_PRIO > 0) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
    };

    int kt = 0;
    for (; kt + 2 < KT; ++kt) {
        phase(kt, 0, false);
        phase(kt, 1, false);
        phase(kt, 2, false);
        phase(kt, 3, false);
    }
    NT_STAMP(2);
    for (; kt < KT; ++kt) {
        phase(kt, 0, true);
        phase(kt, 1, true);
        phase(kt, 2, true);
        phase(kt, 3, true);
    }
#ifndef NT_NO_STAGGER
    if (wr == 0) __builtin_amdgcn_s_barrier();  // match the second wave row's extra barrier
#endif
    NT_STAMP(3);
    pp_epilogue<F>(g, smem, acc, m0, n0, w, l);
    NT_STAMP(4);  // output stores issued (not waited for)
#ifdef NT_PERSIST
    __syncthreads();   // the epilogue's LDS reads are done before the next tile's DMAs land
#endif
    }
#undef NT_STAMP
}

// 3: full-line 256x256 loop (default; buffer-resource LDS-DMAs), 10: the same loop with
// global_load_lds DMAs (rounds 2-4), 2: half-line, 1/0: 128x128.  FEDMI_NT_VARIANT overrides the
// default (A/B runs of whole workloads).
static int nt_default_variant() {
    const char* v = std::getenv("FEDMI_NT_VARIANT");
    return v != nullptr && v[0] != '\0' ? std::atoi(v) : 3;
}
static int g_nt_variant = nt_default_variant();
void gemm_nt_set_variant(int v) { g_nt_variant = v; }
static unsigned long long* g_nt_dbg = nullptr;
void gemm_nt_set_debug(unsigned long long* dbg) { g_nt_dbg = dbg; }

hipError_t gemm_nt_bf16_launch(const NTArgs& g_in, hipStream_t s) {
    NTArgs g = g_in;
    if (g.dbg == nullptr) g.dbg = g_nt_dbg;
    if (g.M % NT_BM || g.N % NT_BN || g.K % NT_BK || g.lda % 8 || g.ldb % 8) return hipErrorInvalidValue;
    if (g_nt_variant == 2 && g.M % NT2_BM == 0 && g.N % NT2_BM == 0 &&
        (g.CbT == nullptr || (g.ldct % 4 == 0 && (reinterpret_cast<uintptr_t>(g.CbT) & 7) == 0)) &&
        (g.mask == nullptr || (g.ldmask % 8 == 0 && (reinterpret_cast<uintptr_t>(g.mask) & 15) == 0)) &&
        (g.Cbf16 == nullptr || (g.ldcb % 8 == 0 && (reinterpret_cast<uintptr_t>(g.Cbf16) & 15) == 0))) {
        const int blocks = (g.M / NT2_BM) * (g.N / NT2_BM);
        hipLaunchKernelGGL(gemm_nt_bf16_pp_kernel, dim3(blocks), dim3(NT2_THREADS), 0, s, g);
        return hipGetLastError();
    }
    if ((g_nt_variant == 3 || g_nt_variant == 10) && g.M % NT2_BM == 0 && g.N % NT2_BM == 0 &&
        (g.CbT == nullptr || (g.ldct % 4 == 0 && (reinterpret_cast<uintptr_t>(g.CbT) & 7) == 0)) &&
        (g.mask == nullptr || (g.ldmask % 8 == 0 && (reinterpret_cast<uintptr_t>(g.mask) & 15) == 0)) &&
        (g.Cbf16 == nullptr || (g.ldcb % 8 == 0 && (reinterpret_cast<uintptr_t>(g.Cbf16) & 15) == 0))) {
        int blocks = (g.M / NT2_BM) * (g.N / NT2_BM);
#ifdef NT_PERSIST
        static int cus = 0;
        if (cus == 0) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8)
                cus = 256;
            cus &= ~7;   // a multiple of 8: the kernel's XCD remap of virtual blocks needs it
        }
        if (blocks > cus) blocks = cus;
#endif
        // The buffer-resource DMAs address a block's operand rows with 32-bit offsets from the
        // block's first row (num_records 0x7fffffff): an out-of-range offset would read zeros
        // silently, so operands whose per-block span (a 256-row tile of A or B, + K) reaches 2^31
        // bytes take the global_load_lds loop (variant 10) instead.
        const size_t span_a = (size_t)NT2_BM * (size_t)g.lda * 2 + (size_t)g.K * 2;
        const size_t span_b = (size_t)NT2_BM * (size_t)g.ldb * 2 + (size_t)g.K * 2;
        const bool glds = g_nt_variant == 10 || span_a >= 0x7fffffffull || span_b >= 0x7fffffffull;
        // the output configurations of the wide client's GEMMs get their own instantiation
        switch (nt_epi_flags(g)) {
#define NT_FL_CASE(F)                                                                                      \
    case F:                                                                                                \
        if (glds) hipLaunchKernelGGL((gemm_nt_bf16_fl_kernel<F, false>), dim3(blocks), dim3(NT2_THREADS), 0, s, g); \
        else hipLaunchKernelGGL((gemm_nt_bf16_fl_kernel<F, true>), dim3(blocks), dim3(NT2_THREADS), 0, s, g);    \
        break;
            NT_FL_CASE(NT_EPI_CB)                                                  // plain bf16 output
            NT_FL_CASE(NT_EPI_CB | NT_EPI_CBT | NT_EPI_BIAS | NT_EPI_RELU)         // hidden-layer forward
            NT_FL_CASE(NT_EPI_CB | NT_EPI_BIAS | NT_EPI_RELU)                      // forward, no transposed copy
            NT_FL_CASE(NT_EPI_CB | NT_EPI_CBT | NT_EPI_MASK)                       // dgrad (ReLU mask)
            NT_FL_CASE(NT_EPI_CB | NT_EPI_CBT | NT_EPI_MASK | NT_EPI_CSUM)         // dgrad + bias gradient
            NT_FL_CASE(NT_EPI_CB | NT_EPI_MASK)                                    // dgrad, no transposed copy
            NT_FL_CASE(NT_EPI_C)                                                   // fp32 output
            NT_FL_CASE(NT_EPI_C | NT_EPI_BETA)                                     // accumulating wgrad
            NT_FL_CASE(NT_EPI_C | NT_EPI_BIAS)                                     // fp32 logits
#undef NT_FL_CASE
            default:
                if (glds) hipLaunchKernelGGL((gemm_nt_bf16_fl_kernel<-1, false>), dim3(blocks), dim3(NT2_THREADS), 0, s, g);
                else hipLaunchKernelGGL((gemm_nt_bf16_fl_kernel<-1, true>), dim3(blocks), dim3(NT2_THREADS), 0, s, g);
                break;
        }
        return hipGetLastError();
    }
    if (g.csum != nullptr) return hipErrorInvalidValue;  // column sums: 256x256 loops only
    const int blocks = (g.M / NT_BM) * (g.N / NT_BN);
    if (g_nt_variant == 0)
        hipLaunchKernelGGL(gemm_nt_bf16_kernel<0>, dim3(blocks), dim3(NT_THREADS), 0, s, g);
    else
        hipLaunchKernelGGL(gemm_nt_bf16_kernel<1>, dim3(blocks), dim3(NT_THREADS), 0, s, g);
    return hipGetLastError();
}

// Transposing bf16 copy: out[c][r] = bf16(in[r][c]) for a [R][C] fp32 matrix (W^T refresh).
__global__ void transpose_bf16_kernel(const float* __restrict__ in, int R, int Cc, int ldi,
                                      __hip_bfloat16* __restrict__ out, int ldo) {
    __shared__ float tile[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
    for (int i = ty; i < 32; i += 8) {
        const int r = r0 + i, c = c0 + tx;
        tile[i][tx] = (r < R && c < Cc) ? in[(size_t)r * ldi + c] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int c = c0 + i, r = r0 + tx;
        if (c < Cc && r < R) out[(size_t)c * ldo + r] = __float2bfloat16(tile[tx][i]);
    }
}

hipError_t transpose_bf16_launch(const float* in, int R, int C, int ldi, void* out, int ldo, hipStream_t s) {
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, s, in, R, C, ldi,
                       reinterpret_cast<__hip_bfloat16*>(out), ldo);
    return hipGetLastError();
}

// Zero-padded bf16 operand: out[r][c] = bf16(in[r*rs + c*cs]) for c < C, 0 for C <= c < ldo.
// Pads the K = 14 input features / the C = 2 logit deltas to K = 64 so the layer-0 forward and
// the head's dgrad run on the NT GEMM (with their fused bias/ReLU/mask and transposed outputs)
// instead of the generic kernel + an fp32 scratch + a transpose pass; with cs != 1 it also
// transposes (the head's W^T).
__global__ void pad_bf16_kernel(const float* __restrict__ in, int R, int C, long long rs, long long cs,
                                __hip_bfloat16* __restrict__ out, int ldo) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)R * ldo) return;
    const int r = (int)(i / ldo), c = (int)(i % ldo);
    out[i] = __float2bfloat16(c < C ? in[r * rs + c * cs] : 0.f);
}

hipError_t pad_bf16_launch(const float* in, int R, int C, long long rs, long long cs, void* out, int ldo,
                           hipStream_t s) {
    if (C > ldo) return hipErrorInvalidValue;
    const size_t n = (size_t)R * ldo;
    hipLaunchKernelGGL(pad_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, R, C, rs, cs,
                       reinterpret_cast<__hip_bfloat16*>(out), ldo);
    return hipGetLastError();
}

// Bias gradient from a transposed bf16 delta: out[n] (+)= sum_r dT[n][r], one wave per row,
// 16-byte loads, fixed-order reduction (deterministic across runs).
__global__ void __launch_bounds__(256) rowsum_bf16_kernel(const __hip_bfloat16* __restrict__ dT, int Nrows, int M,
                                                          int ld, float* __restrict__ out, float beta) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= Nrows) return;
    const __hip_bfloat16* p = dT + (size_t)row * ld;
    float acc = 0.f;
    for (int c = lane * 8; c < M; c += 512) {
        const uint4 u = *reinterpret_cast<const uint4*>(p + c);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) out[row] = beta != 0.f ? beta * out[row] + acc : acc;
}

hipError_t rowsum_bf16_launch(const void* dT, int Nrows, int M, int ld, float* out, float beta, hipStream_t s) {
    if (M % 8 || ld % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rowsum_bf16_kernel, dim3((Nrows + 3) / 4), dim3(256), 0, s,
                       reinterpret_cast<const __hip_bfloat16*>(dT), Nrows, M, ld, out, beta);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Skinny weight gradient over a long contraction (the wide MLP's layer 0, 14 input features, and
// its logits head, C classes), bandwidth-bound:  out = beta*out + sum_rows S[row][c] * W[row][n]
// for c < C, n < Nw.  W: [rows][ldw] bf16 (the wide side: 4096 deltas or activations), S:
// [rows][lds] bf16 (the skinny side, row-uniform, so the compiler reads it with scalar loads).
// A thread owns 8 consecutive n (one 16-byte load per row) x C fp32 accumulators; a block of 256
// threads spans 2048 columns; blockIdx.y = z contracts rows [z*rc, (z+1)*rc) into slab[z], and
// splitk_reduce folds the slabs in fixed order (deterministic).  TRANS = 0 writes out[c][n]
// (ld Nw: the head's dW[C][H]), TRANS = 1 out[n][c] (ld C: layer 0's dW[H][14]).  Replaces the
// MFMA tile GEMM there, whose 64-row tiles over C <= 14 wasted the matrix core and streamed the
// wide operand at ~1.3 TB/s.  BIAS = 1 also sums the wide operand's columns (layer 0's bias
// gradient, sum over rows of dZ0) into slab[z][C*Nw + n], from the same loads.
template <int C, int TRANS, int BIAS>
__global__ void __launch_bounds__(256)
skinny_wgrad_kernel(const __hip_bfloat16* __restrict__ W, int ldw, int Nw, const __hip_bfloat16* __restrict__ S,
                    int lds, int rows, int rc, float* __restrict__ slab) {
    const int n0 = (blockIdx.x * 256 + threadIdx.x) * 8;
    const int z = blockIdx.y;
    const int r0 = z * rc, r1 = min(rows, r0 + rc);
    float acc[C][8], bsum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[e] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][e] = 0.f;
    if (n0 < Nw) {
#pragma unroll 4
        for (int r = r0; r < r1; ++r) {
            const uint4 wv = *reinterpret_cast<const uint4*>(W + (size_t)r * ldw + n0);
            const uint32_t wu[4] = {wv.x, wv.y, wv.z, wv.w};
            float wf[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                wf[2 * q] = __uint_as_float(wu[q] << 16);
                wf[2 * q + 1] = __uint_as_float(wu[q] & 0xffff0000u);
            }
            if (BIAS) {
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum[e] += wf[e];
            }
            const __hip_bfloat16* srow = S + (size_t)r * lds;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float sc = __bfloat162float(srow[c]);
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[c][e] = fmaf(sc, wf[e], acc[c][e]);
            }
        }
    }
    if (n0 >= Nw) return;
    float* out = slab + (size_t)z * (C + BIAS) * Nw;
    if (BIAS) {
        float4* o = reinterpret_cast<float4*>(out + (size_t)C * Nw + n0);
        o[0] = make_float4(bsum[0], bsum[1], bsum[2], bsum[3]);
        o[1] = make_float4(bsum[4], bsum[5], bsum[6], bsum[7]);
    }
    if (TRANS == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            float4* o = reinterpret_cast<float4*>(out + (size_t)c * Nw + n0);
            o[0] = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
            o[1] = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
        }
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int c = 0; c < C; ++c) out[(size_t)(n0 + e) * C + c] = acc[c][e];
    }
}

hipError_t skinny_wgrad_launch(const void* W, int ldw, int Nw, const void* S, int lds, int C, int rows, int trans,
                               int splits, float* slab, float* out, float beta, float* bias_out, hipStream_t s) {
    if (Nw % 8 || ldw % 8 || (reinterpret_cast<uintptr_t>(W) & 15) || splits < 1 || lds < C) return hipErrorInvalidValue;
    const int rc = (rows + splits - 1) / splits;
    const dim3 grid((unsigned)((Nw / 8 + 255) / 256), (unsigned)splits);
    const __hip_bfloat16* w = reinterpret_cast<const __hip_bfloat16*>(W);
    const __hip_bfloat16* sk = reinterpret_cast<const __hip_bfloat16*>(S);
    const int nb = bias_out != nullptr ? 1 : 0;
    if (C == 2 && trans == 0 && !nb)
        hipLaunchKernelGGL((skinny_wgrad_kernel<2, 0, 0>), grid, dim3(256), 0, s, w, ldw, Nw, sk, lds, rows, rc, slab);
    else if (C == 14 && trans == 1 && !nb)
        hipLaunchKernelGGL((skinny_wgrad_kernel<14, 1, 0>), grid, dim3(256), 0, s, w, ldw, Nw, sk, lds, rows, rc, slab);
    else if (C == 14 && trans == 1)
        hipLaunchKernelGGL((skinny_wgrad_kernel<14, 1, 1>), grid, dim3(256), 0, s, w, ldw, Nw, sk, lds, rows, rc, slab);
    else
        return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t stride = (size_t)(C + nb) * Nw;
    e = splitk_reduce_launch(slab, stride, splits, out, (size_t)C * Nw, beta, s);
    if (e != hipSuccess || !nb) return e;
    return splitk_reduce_launch(slab + (size_t)C * Nw, stride, splits, bias_out, (size_t)Nw, beta, s);
}
