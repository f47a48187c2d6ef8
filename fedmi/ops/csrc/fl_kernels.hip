// Fused federated-round kernels for gfx950 (MI355X / CDNA4).
//
// The reference round (FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:130-201)
// is ~20 ATen launches + 6 H2D/D2H copies + pickled MPI gather/bcast per round.  Here the
// classic round is three kernels and one all-reduce on one stream:
//
//   fl_train  : per-workgroup fwd + CE + bwd over R rows with the parameter image AND
//               activations in LDS; dense weight-gradient partials -> slab row (non-temporal)
//                                                                  (K2-K17)
//   fl_adam   : fold of the previous round's metrics (history, early stop, live decision);
//               wide deterministic slab reduction (16 waves per 64 parameters) + Adam
//               (+L2, +FedProx) + StepLR; writes the local image and the pre-scaled (n_i/N)
//               FedAvg contribution                                (K18, K22)
//   fl_eval   : forward of the post-step local model on the local shard, argmax and the
//               C x C confusion matrix into this rank's tail slot  (K20, Q2)
//   allreduce : one SUM over [image*n_i/N | per-rank tails] = gather + average + bcast of
//               weights, sizes, metrics and stop signal in one collective (§2.4)
//
// and the steady-state rounds are TWO kernels (fl_common.h FL_EVAL_*): with one client the
// train kernel scores the previous round's model from its own forward pass; with several
// the bf16 train kernel scores it with a second forward pass (lagged) and the FedAvg runs
// inside fl_adam (one-shot xGMI chunk exchange, peer_device.h).
//
// GEMM-shaped work runs on the f32-input MFMA (v_mfma_f32_16x16x4_f32: exact f32 fma chain;
// the reference trains in fp32).  Work items are 16-wide column tiles spread over the 16
// waves of a 1024-thread workgroup (fl_device.h FL_THREADS); a wave keeps one accumulator
// per 16-row tile so a B fragment is read once per k and reused RT times, and the next
// 16-deep k chunk is loaded
// while the current one is multiplied.  The skinny classifier head (C outputs) runs on the
// VALU with a fixed-order split-K shuffle reduction.
#include "fl_common.h"
#include "fl_device.h"
#include "peer_device.h"
#include <math.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------
// Block-cooperative GEMM pieces (operand maps of 16x16x4 f32 MFMA:
//   A lane l -> A[l&15][l>>4], B lane l -> B[l>>4][l&15], C/D: col l&15, row 4(l>>4)+j).
// The contraction order is free, so k is permuted: in a 16-deep chunk q, MFMA step j takes
// k = 16q + 4*lg + j from lane group lg.  A lane then owns 4 CONSECUTIVE k, i.e. one 16-byte
// ds_read_b128 per operand wherever k runs along an LDS row.  All loads of a chunk are issued
// before its MFMAs (sched_barrier), so LDS latency overlaps the matrix pipe.
//
// LDS chunk swizzle: every fp32 LDS matrix (activations, deltas, logits, and the weight rows,
// already swizzled in the parameter image, fl_common.h) keeps logical column k <
// roundup16(width) of row r at column k ^ fl_swz(r), i.e. the
// 4-float chunks of rows 4..11 (mod 16) trade places in pairs (pad columns stay put).  A b128
// operand read -- lane (row lr, chunk lg) -- covers 8 rows at chunk g and 8 rows at chunk g ^ 1
// in each of the four gfx950 b128 lane groups; with row strides 4 mod 8 floats those collided
// on one 16-byte bank slot (4 extra LDS cycles per read: 0.55 conflict cycles per LDS
// instruction measured, profiles/pmc_summary_r3s2.txt), with the swizzle all 16 land on distinct
// slots (tools/bank_fp32.py models both).  b32 accesses of 16 consecutive columns of a row touch
// the same banks as before.  Rows 16t + 4g + j of a C/D fragment share fl_swz(4g): one per-lane
// constant (fl_swz_lg) for every output / b32 access.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int fl_swz_lg(int lg) { return (lg == 1 || lg == 2) ? 4 : 0; }  // = fl_swz(4 lg + j)

__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float f4(const float4& v, int j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// out[r][n] = act(sum_k in[r][k] W[n][k] + bias[n]) for all R rows; columns
// [N, roundup16(N)) come out 0 (zero image rows + zero bias padding).
template <int RT>
__device__ void fwd_layer_mfma(const float* w, int ldw, const float* bias, int K, int N, const float* in,
                               int ld_in, float* out, int ld_out, bool relu) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    const int ntiles = (N + 15) >> 4;
    const int kchunks = (K + 15) >> 4;
    for (int nt = wave; nt < ntiles; nt += FL_WAVES) {
        const int n = nt * 16 + lr;
        const int ck = (4 * lg) ^ fl_swz(lr);  // operand chunk (rows n and lr + 16 rt: fl_swz(lr))
        const float* wr = w + n * ldw + ck;
        const float* ar = in + lr * ld_in + ck;
        f32x4 acc[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        float4 bc = lds4(wr), ac[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) ac[rt] = lds4(ar + rt * 16 * ld_in);
        // the last chunk's steps j >= K - 16q are all-padding when K - 16q <= 4 (step j of lane
        // group g takes k = 16q + 4g + j): skipped -- they would add exact zeros (a (50, 200) layer
        // runs 14 of 16 steps)
        const int klast = K - 16 * (kchunks - 1);
        for (int q = 0; q < kchunks; ++q) {
            const int qn = (q + 1 < kchunks) ? q + 1 : q;  // prefetch (last: harmless reload)
            const float4 bn = lds4(wr + 16 * qn);
            float4 an[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) an[rt] = lds4(ar + rt * 16 * ld_in + 16 * qn);
            __builtin_amdgcn_sched_barrier(0);
            const int jmax = (q + 1 < kchunks || klast > 4) ? 4 : klast;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < jmax)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma_f32(f4(ac[rt], j), f4(bc, j), acc[rt]);
            __builtin_amdgcn_sched_barrier(0);
            bc = bn;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) ac[rt] = an[rt];
        }
        const float bv = bias[n];
        const int ns = n ^ fl_swz_lg(lg);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[rt][j] + bv;
                if (relu) v = fmaxf(v, 0.f);
                out[(rt * 16 + lg * 4 + j) * ld_out + ns] = v;
            }
    }
}

// Skinny head on the VALU: z[r][c] = bias[c] + sum_k in[r][k] W[c][k] for R*C <= 128.
// T threads per output (power of 2), fixed-order xor-shuffle reduction (deterministic).
template <int RT>
__device__ void fwd_head_valu(const float* w, int ldw, const float* bias, int K, int C, const float* in,
                              int ld_in, float* out, int ld_out) {
    const int R = RT * 16;
    const int nout = R * C;
    int T = FL_THREADS / nout;
    T = T >= 64 ? 64 : (T >= 32 ? 32 : (T >= 16 ? 16 : (T >= 8 ? 8 : (T >= 4 ? 4 : (T >= 2 ? 2 : 1)))));
    const int K16 = (K + 15) & ~15;  // zero padded in both operands
    for (int base = 0; base < nout * T; base += FL_THREADS) {
        const int gid = base + threadIdx.x;
        const int o = gid / T, part = gid - o * T;
        const int oc = o < nout ? o : nout - 1;
        const int r = oc / C, c = oc - r * C;
        const float* ar = in + r * ld_in;
        const float* wr = w + c * ldw;
        const int sa = fl_swz(r), sw = fl_swz(c);
        float s0 = 0.f, s1 = 0.f;
        // 4 consecutive k per thread per step: float4 reads
        int k = 4 * part;
        for (; k + 4 * T < K16; k += 8 * T) {
            const float4 a0 = lds4(ar + (k ^ sa)), w0 = lds4(wr + (k ^ sw));
            const float4 a1 = lds4(ar + ((k + 4 * T) ^ sa)), w1 = lds4(wr + ((k + 4 * T) ^ sw));
            s0 = fmaf(a0.x, w0.x, s0); s0 = fmaf(a0.y, w0.y, s0); s0 = fmaf(a0.z, w0.z, s0); s0 = fmaf(a0.w, w0.w, s0);
            s1 = fmaf(a1.x, w1.x, s1); s1 = fmaf(a1.y, w1.y, s1); s1 = fmaf(a1.z, w1.z, s1); s1 = fmaf(a1.w, w1.w, s1);
        }
        if (k < K16) {
            const float4 a0 = lds4(ar + (k ^ sa)), w0 = lds4(wr + (k ^ sw));
            s0 = fmaf(a0.x, w0.x, s0); s0 = fmaf(a0.y, w0.y, s0); s0 = fmaf(a0.z, w0.z, s0); s0 = fmaf(a0.w, w0.w, s0);
        }
        float s = s0 + s1;
        for (int off = 1; off < T; off <<= 1) s += __shfl_xor(s, off, 64);
        if (o < nout && part == 0) out[r * ld_out + (c ^ sa)] = s + bias[c];
    }
    const int Cp = (C + 15) & ~15;  // zero padded columns [C, roundup16(C))
    for (int e = threadIdx.x; e < R * (Cp - C); e += FL_THREADS) {
        const int r = e / (Cp - C), c = C + (e - r * (Cp - C));
        out[r * ld_out + (c ^ fl_swz(r))] = 0.f;
    }
}

// Waves that take wgrad tiles in the backward phase of layer l (the fp32 twin of
// wgrad_waves_bf16): the dgrad items (one per 16 input columns, handed out from the last wave
// down) are chains of ochunks dependent 16-deep steps; when they are long (the 50 -> 200 layer:
// 4 items of 13 steps, 104 MFMAs each) their waves take no wgrad tiles -- which otherwise
// stacked in front of the chain on the same waves (stamps: the last wave started its dgrad
// 4.8 us into the phase, then ran 3.2 us) -- and the phase ends with an LDS arrival count of
// those waves instead of a barrier (fl_train_body.inc).  Only the work-to-wave map changes.
__device__ __forceinline__ int wgrad_waves_fp32(int K, int N, int l) {
    const int items = l > 0 ? (K + 15) >> 4 : 0;
    const int chunks = (N + 15) >> 4;
    return (items > 0 && chunks >= 4 && 2 * items <= FL_WAVES) ? FL_WAVES - items : FL_WAVES;
}

// dH[r][i] = (sum_o dZ[r][o] W[o][i]) * (act[r][i] > 0) -> out (separate buffer, so the
// same phase can run the layer's wgrad, which reads act).  Item = 16-column tile of dH (all
// R rows); B fragment W[o][i] reused across the RT rows.  Items are handed out from the
// LAST wave down, so they pair with the wgrad tiles handed out from wave 0 up.
template <int RT>
__device__ void dgrad_layer(const float* w, int ldw, int K, int N, const float* dz, int ld_z, const float* act,
                            int ld_a, float* out) {
    const int wave = (FL_WAVES - 1) - (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    const int itiles = (K + 15) >> 4;
    const int ochunks = (N + 15) >> 4;
    // long dgrad chains (their own waves, wgrad_waves_fp32) issue ahead of the wgrad tiles that
    // share their SIMDs: the chain is the phase's critical path (fp32 round 29.5 -> 28.6 us,
    // profiles/fp32_backward_r4.log)
    const bool prio = ochunks >= 4 && wave < itiles;
    if (prio) __builtin_amdgcn_s_setprio(2);
    for (int it = wave; it < itiles; it += FL_WAVES) {
        const int i = it * 16 + lr;
        const int is = i ^ fl_swz_lg(lg);                        // column i of rows 16t + 4lg + j
        const float* wc = w + 4 * lg * ldw + is;                 // B: W[16q + 4lg + j][i]
        const float* ar = dz + lr * ld_z + ((4 * lg) ^ fl_swz(lr));  // A: dZ[r][16q + 4lg + j]
        f32x4 acc[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        float bc[4];
        float4 ac[RT];
#pragma unroll
        for (int j = 0; j < 4; ++j) bc[j] = wc[j * ldw];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) ac[rt] = lds4(ar + rt * 16 * ld_z);
        for (int q = 0; q < ochunks; ++q) {
            const int qn = (q + 1 < ochunks) ? q + 1 : q;
            float bn[4];
            float4 an[RT];
#pragma unroll
            for (int j = 0; j < 4; ++j) bn[j] = wc[(16 * qn + j) * ldw];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) an[rt] = lds4(ar + rt * 16 * ld_z + 16 * qn);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma_f32(f4(ac[rt], j), bc[j], acc[rt]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 4; ++j) bc[j] = bn[j];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) ac[rt] = an[rt];
        }
        const bool ivalid = i < K;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = (rt * 16 + lg * 4 + j) * ld_a + is;
                out[o] = (ivalid && act[o] > 0.f) ? acc[rt][j] : 0.f;
            }
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
}

// dW[o][i] = sum_r dZ[r][o] act[r][i] over the block's rows -> gW ([N][K] dense, global);
// gb[o] = sum_r dZ[r][o].  Two output tiles per wave are interleaved (independent chains);
// row r = 16q + 4lg + j of chunk q feeds MFMA step j of lane group lg.
// Tiles go to `nw` waves: waves [0, nw) from wave 0 up, or (`top`) the last nw waves from the
// top down; waves outside them take none (they run a long dgrad chain, wgrad_waves_fp32).  A
// wave's lone last tile runs alone (no duplicate second chain on the MFMA pipe).
template <int RT>
__device__ void wgrad_layer(int K, int N, const float* dz, int ld_z, const float* act, int ld_a,
                            float* __restrict__ gW, float* __restrict__ gb, int nw = FL_WAVES, bool top = false) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    const int otiles = (N + 15) >> 4, itiles = (K + 15) >> 4;
    const int ntile = otiles * itiles;
    const int w = top ? FL_WAVES - 1 - wave : wave;
    for (int t0 = w < nw ? w : ntile; t0 < ntile; t0 += 2 * nw) {
        const int t1raw = t0 + nw;
        const bool has1 = t1raw < ntile;
        const int t1 = has1 ? t1raw : t0;
        const int ot0 = t0 / itiles, it0 = t0 - ot0 * itiles;
        const int ot1 = t1 / itiles, it1 = t1 - ot1 * itiles;
        const int ls = lr ^ fl_swz_lg(lg);  // columns of rows 16q + 4lg + j
        const float* ap0 = dz + 4 * lg * ld_z + ot0 * 16 + ls;
        const float* bp0 = act + 4 * lg * ld_a + it0 * 16 + ls;
        const float* ap1 = dz + 4 * lg * ld_z + ot1 * 16 + ls;
        const float* bp1 = act + 4 * lg * ld_a + it1 * 16 + ls;
        float a0[RT * 4], b0[RT * 4], a1[RT * 4], b1[RT * 4];
#pragma unroll
        for (int q = 0; q < RT; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int s = 4 * q + j;
                a0[s] = ap0[(16 * q + j) * ld_z]; b0[s] = bp0[(16 * q + j) * ld_a];
                a1[s] = ap1[(16 * q + j) * ld_z]; b1[s] = bp1[(16 * q + j) * ld_a];
            }
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc0 = (f32x4){0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
        if (has1) {  // (wave-uniform)
#pragma unroll
            for (int s = 0; s < RT * 4; ++s) {
                acc0 = mfma_f32(a0[s], b0[s], acc0);
                acc1 = mfma_f32(a1[s], b1[s], acc1);
            }
        } else {
#pragma unroll
            for (int s = 0; s < RT * 4; ++s) acc0 = mfma_f32(a0[s], b0[s], acc0);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int i0 = it0 * 16 + lr, i1 = it1 * 16 + lr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o0 = ot0 * 16 + lg * 4 + j, o1 = ot1 * 16 + lg * 4 + j;
            if (i0 < K && o0 < N) slab_store(&gW[o0 * K + i0], acc0[j]);
            if (has1 && i1 < K && o1 < N) slab_store(&gW[o1 * K + i1], acc1[j]);
        }
    }
    for (int o = threadIdx.x; o < N; o += FL_THREADS) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int r = 0; r < RT * 16; r += 2) {
            s0 += dz[r * ld_z + (o ^ fl_swz(r))];
            s1 += dz[(r + 1) * ld_z + (o ^ fl_swz(r + 1))];
        }
        slab_store(&gb[o], s0 + s1);
    }
}

template <int RT>
__device__ void stage_rows(const float* __restrict__ X, int n_rows, int F, int row0, float* xs, int ld) {
    const int F16 = (F + 15) & ~15;
    for (int e = threadIdx.x; e < RT * 16 * ld; e += FL_THREADS) {
        const int r = e / ld, cs = e - r * ld;
        const int c = cs < F16 ? cs ^ fl_swz(r) : cs;  // logical column stored at cs
        const int row = row0 + r;
        const bool ok = row < n_rows && c < F;
        const float v = X[(size_t)(ok ? row : 0) * F + (ok ? c : 0)];  // unpredicated load
        xs[e] = ok ? v : 0.f;
    }
}

// The global parameter image is bit-identical to the LDS image (weight rows already swizzled,
// fl_common.h): one float4 copy.
__device__ __forceinline__ void stage_image(const MLPDesc& d, const float* __restrict__ params, float* li) {
    const float4* src = reinterpret_cast<const float4*>(params);
    float4* dst = reinterpret_cast<float4*>(li);
    const int n4 = d.Pimg >> 2;
    for (int e = threadIdx.x; e < n4; e += FL_THREADS) dst[e] = src[e];
}

template <int RT>
__device__ void forward_block(const MLPDesc& d, float* acts, const float* li, unsigned long long* dbg = nullptr) {
    for (int l = 0; l < d.L; ++l) {
        if (dbg != nullptr && threadIdx.x == 0) dbg[blockIdx.x * 16 + 10 + l] = __builtin_amdgcn_s_memrealtime();
        const int K = d.dim[l], N = d.dim[l + 1];
        const float* w = li + d.iw_off[l];
        const float* bias = li + d.ib_off[l];
        if (l + 1 == d.L && RT * 16 * N <= 128)
            fwd_head_valu<RT>(w, fl_ldw(K), bias, K, N, acts + d.act_off[l], d.ld[l], acts + d.act_off[l + 1],
                              d.ld[l + 1]);
        else
            fwd_layer_mfma<RT>(w, fl_ldw(K), bias, K, N, acts + d.act_off[l], d.ld[l], acts + d.act_off[l + 1],
                               d.ld[l + 1], l + 1 < d.L);
        lds_barrier();
    }
}

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------
// Kernel body shared by the single-engine and trial-batch entry points (fl_train_body.inc).
template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_train_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pg,
                const FLState* __restrict__ st_in, FLState* __restrict__ st_out, int local_step, int mode,
                float* __restrict__ cm_out, int fold_mask) {
#include "fl_train_body.inc"
}

template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_train_batch_kernel(MLPDesc d, const FLTrialDesc* __restrict__ T, FLSel pg_sel, FLSel si_sel, FLSel so_sel,
                      int local_step, int mode, FLSel cm_sel, int fold_mask) {
    const FLTrialDesc& t = T[blockIdx.y];
    const FLConfig c = t.c;
    const FLBuffers b = t.b;
    const float* __restrict__ pg = reinterpret_cast<const float*>(fl_sel(t, pg_sel));
    const FLState* __restrict__ st_in = reinterpret_cast<const FLState*>(fl_sel(t, si_sel));
    FLState* __restrict__ st_out = reinterpret_cast<FLState*>(fl_sel(t, so_sel));
    float* __restrict__ cm_out = reinterpret_cast<float*>(fl_sel(t, cm_sel));
#include "fl_train_body.inc"
}

#include "fl_adam.h"

// Block 0 is the tail block (dispatched first: with the in-kernel fold every other block may
// wait for its lag chunk); blocks 1.. own 64 dense parameters each.
// Kernel body shared by the single-engine and trial-batch entry points (fl_adam_body.inc).
__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
               const float* __restrict__ anchor, float* __restrict__ comm,
               const FLState* __restrict__ st, int local_step, MLPDescB e, int pack,
               FLState* __restrict__ st_out, int fold, int tail_a, int fold_mask, PeerArgs pa, int xchg,
               int afold) {
#define ADAM_PA_LL (pa.ll != nullptr)
#include "fl_adam_body.inc"
#undef ADAM_PA_LL
}

// The general body on a VIRTUAL grid, for the publish / wait / pull exchange (FEDMI_PEER_LL=0)
// of ranks that SHARE a GPU: the counterpart of fl_adam_ll_grid_kernel (fl_adam_local.hip; same
// block order, same deadlock-freedom argument, bit-identical values).  Without it a shared GPU
// cannot hold every rank's spinning pull grid at once (8 ranks stalled, profiles/plane_companions_r5.log).
__device__ __forceinline__ void fl_adam_vblock(const int adam_blk, const MLPDesc& d, const FLConfig& c,
                                               const FLBuffers& b, const float* __restrict__ pin,
                                               const float* __restrict__ anchor, float* __restrict__ comm,
                                               const FLState* __restrict__ st, int local_step, const MLPDescB& e,
                                               int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                                               int fold_mask, const PeerArgs& pa, int xchg, int afold) {
#define ADAM_PA_LL (pa.ll != nullptr)
#define ADAM_BLK adam_blk
#include "fl_adam_body.inc"
#undef ADAM_BLK
#undef ADAM_PA_LL
}

__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_grid_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                    const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                    int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                    int fold_mask, PeerArgs pa, int xchg, int afold, int n_vblocks) {
    for (int vb = blockIdx.x; vb < n_vblocks; vb += gridDim.x) {
        fl_adam_vblock(vb, d, c, b, pin, anchor, comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask, pa,
                       xchg, afold);
        __syncthreads();  // the block's LDS (partials, state) is free before the next virtual block
    }
}

// (the trial-batch Adam kernel lives in fl_adam_batch.hip: 4-wave blocks, same canonical sums)

// Local evaluation of the post-step model on the local shard (C:148, C:75-91): forward,
// argmax, confusion counts into this rank's tail (exact: integer-valued fp32 < 2^24).
template <int RT>
__device__ void eval_rows(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* __restrict__ params,
                          float* __restrict__ cm_out, int blk, float* lds) {
    __shared__ int cm_s[FL_MAX_CLASSES * FL_MAX_CLASSES];
    const int R = RT * 16;
    const int row0 = blk * R;
    const int C = d.dim[d.L];
    float* acts = lds;
    float* li = lds + d.img_lds;
    FL_STAMP(0);
    for (int e = threadIdx.x; e < C * C; e += FL_THREADS) cm_s[e] = 0;
    // labels are needed only after the forward pass: issue the load now
    const int ylab = (threadIdx.x < R) ? b.y[min(row0 + (int)threadIdx.x, c.n_rows - 1)] : 0;
    stage_image(d, params, li);
    stage_rows<RT>(b.X, c.n_rows, d.dim[0], row0, acts + d.act_off[0], d.ld[0]);
    lds_barrier();
    FL_STAMP(1);
    forward_block<RT>(d, acts, li);
    FL_STAMP(2);
    if (threadIdx.x < R) {
        const int r = threadIdx.x, row = row0 + r;
        if (row < c.n_rows) {
            const float* zr = acts + d.act_off[d.L] + r * d.ld[d.L];
            const int sr = fl_swz(r);
            int best = 0;
            float bv = zr[sr];
            for (int k = 1; k < C; ++k)
                if (zr[k ^ sr] > bv) { bv = zr[k ^ sr]; best = k; }
            atomicAdd(&cm_s[ylab * C + best], 1);
        }
    }
    lds_barrier();
    for (int e = threadIdx.x; e < C * C; e += FL_THREADS)
        if (cm_s[e]) atomicAdd(&cm_out[e], (float)cm_s[e]);
    FL_STAMP(15);
}

template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_eval_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ params,
               float* __restrict__ cm_out, const FLState* __restrict__ st) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (st != nullptr && !st->live) return;
    eval_rows<RT>(d, c, b, params, cm_out, blockIdx.x, lds);
}

// Local evaluation + FedAvg in one kernel (world > 1, one-shot xGMI all-reduce); see
// fl_eval_fedavg_bf16_kernel.
template <int RT>
__global__ void __launch_bounds__(FL_THREADS, 8)  // 8 waves/SIMD = two workgroups per CU: one resident wave of blocks
fl_eval_fedavg_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ params,
                      float* __restrict__ cm_out, const FLState* __restrict__ st, PeerArgs a, PeerPack pk, int n_ar) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const unsigned target = peer_target(a);
    if ((int)blockIdx.x < n_ar) {
        peer_fused_reduce(a, pk, target, blockIdx.x, n_ar);
        peer_finish(a, target, n_ar);
    } else {
        if (st->live) eval_rows<RT>(d, c, b, params, cm_out, blockIdx.x - n_ar, lds);
        peer_eval_done(a, target, blockIdx.x - n_ar);
    }
}

__global__ void fl_finalize_kernel(MLPDesc d, FLConfig c, FLBuffers b, float* __restrict__ pg,
                                   const FLState* __restrict__ st_in, FLState* __restrict__ st_out, int mask,
                                   const float* __restrict__ prev_out) {
    if (blockIdx.x != 0) return;
    const FLState Sin = *st_in;
    FLState S = finalize_state(d, c, b, pg, Sin, true, mask);
    // a stop found one round late (fold of region A, FLState::late): the last round ran past it;
    // its output image is replaced by the round before's, still intact in the other buffer
    int late = (threadIdx.x == 0 && !Sin.stopped && S.stopped && S.stop_round < Sin.next_round) ? 1 : 0;
    late = __shfl(late, 0, 64);
    if (late && prev_out != nullptr)
        for (int i = threadIdx.x * 4; i < d.Pimg; i += 64 * 4)
            *reinterpret_cast<float4*>(pg + i) = *reinterpret_cast<const float4*>(prev_out + i);
    if (late && b.undo != nullptr) {
        // ... and the local model, Adam moments and packed local image of that round too
        float* const dst[3] = {b.local, b.m, b.v};
        for (int a = 0; a < 3; ++a)
            for (int i = threadIdx.x * 4; i < d.Pimg; i += 64 * 4)
                *reinterpret_cast<float4*>(dst[a] + i) = *reinterpret_cast<const float4*>(b.undo + a * d.Pimg + i);
        if (b.pk_local != nullptr) {
            const char* src = reinterpret_cast<const char*>(b.undo + 3 * d.Pimg);
            for (int i = threadIdx.x * 4; i < b.undo_pk_bytes; i += 64 * 4)
                *reinterpret_cast<uint32_t*>(b.pk_local + i) = *reinterpret_cast<const uint32_t*>(src + i);
        }
    }
    if (threadIdx.x != 0) return;
    S.live = 0;
    S.late = late;
    *st_out = S;
}

template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_eval_batch_kernel(MLPDesc d, const FLTrialDesc* __restrict__ T, FLSel params, FLSel comm, FLSel st) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const FLTrialDesc& t = T[blockIdx.y];
    const FLState* s = reinterpret_cast<const FLState*>(fl_sel(t, st));
    if (s != nullptr && !s->live) return;
    float* cm = reinterpret_cast<float*>(fl_sel(t, comm)) + t.c.tail_off + t.c.rank * t.c.tail_stride;
    eval_rows<RT>(d, t.c, t.b, reinterpret_cast<const float*>(fl_sel(t, params)), cm, blockIdx.x, lds);
}

__global__ void fl_finalize_batch_kernel(MLPDesc d, const FLTrialDesc* __restrict__ T, FLSel pg, FLSel si, FLSel so,
                                         int mask) {
    const FLTrialDesc& t = T[blockIdx.y];
    FLState S = finalize_state(d, t.c, t.b, reinterpret_cast<const float*>(fl_sel(t, pg)),
                               *reinterpret_cast<const FLState*>(fl_sel(t, si)), true, mask);
    if (threadIdx.x != 0) return;
    S.live = 0;
    *reinterpret_cast<FLState*>(fl_sel(t, so)) = S;
}

// ---------------------------------------------------------------------------------------
// Synthetic income-shaped rows: Philox4x32-10 counter-based RNG, one row per thread.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                             uint32_t k0, uint32_t k1) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
}

__device__ __forceinline__ uint4 philox4x32(uint64_t ctr, uint32_t sub, uint64_t key) {
    uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = sub, c3 = 0x9E3779B9u;
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        philox_round(c0, c1, c2, c3, k0, k1);
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ float u01(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__global__ void fl_synth_kernel(float* __restrict__ X, int* __restrict__ y, long long n, int F,
                                unsigned long long seed, unsigned long long row_offset,
                                const float* __restrict__ w1, const float* __restrict__ w2, int H,
                                float label_noise) {
    const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    const uint64_t gid = row_offset + (uint64_t)row;
    float x[32];
    const int cards[8] = {7, 16, 7, 14, 6, 5, 2, 40};
    for (int col = 0; col < F; ++col) {
        const uint4 r2 = philox4x32(gid, (uint32_t)col, seed);
        const float u1 = u01(r2.x), u2 = u01(r2.y);
        float val;
        if (col < 6) {
            val = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
        } else {
            const int card = cards[(col - 6) & 7];
            const float code = floorf(u01(r2.z) * card);
            const float mean = 0.5f * (card - 1), sd = sqrtf((card * card - 1) / 12.f);
            val = (code - mean) / sd;
        }
        x[col] = val;
        X[(size_t)row * F + col] = val;
    }
    float score = 0.f;
    for (int h = 0; h < H; ++h) {
        float a = 0.f;
        for (int f = 0; f < F; ++f) a += w1[h * F + f] * x[f];
        score += w2[h] * fmaxf(a, 0.f);
    }
    int label = score > w2[H] ? 1 : 0;  // w2[H] holds the balancing threshold
    // label noise: flip with probability `label_noise` (its own Philox stream, column F), so the
    // synthetic task has a Bayes accuracy like the income table's (~0.85) instead of 1
    if (label_noise > 0.f && u01(philox4x32(gid, (uint32_t)F, seed).w) < label_noise) label ^= 1;
    y[row] = label;
}

// ---------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------
static inline int nblocks(int n, int R) { return (n + R - 1) / R; }
static inline size_t lds_bytes(const MLPDesc& d) { return (size_t)d.lds_floats * sizeof(float); }

template <int RT>
static hipError_t launch_train_rt(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                                  const float* pg, const FLState* si, FLState* so, int ls, hipStream_t s,
                                  int mode, float* cm_out, int fold_mask) {
    hipLaunchKernelGGL(fl_train_kernel<RT>, dim3(c.n_slabs), dim3(FL_THREADS), lds_bytes(d), s, d, c, b, pg, si,
                       so, ls, mode, cm_out, fold_mask);
    return hipGetLastError();
}

hipError_t fl_launch_train(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pg,
                           const FLState* si, FLState* so, int ls, hipStream_t s, int mode, float* cm_out,
                           int fold_mask) {
    if (mode == FL_EVAL_FUSED && cm_out == nullptr) return hipErrorInvalidValue;
    if (mode == FL_EVAL_LAGGED) return hipErrorInvalidValue;  // bf16 kernels only
    switch (c.R) {
        case 16: return launch_train_rt<1>(d, c, b, pg, si, so, ls, s, mode, cm_out, fold_mask);
        case 32: return launch_train_rt<2>(d, c, b, pg, si, so, ls, s, mode, cm_out, fold_mask);
        default: return hipErrorInvalidValue;
    }
}

hipError_t fl_launch_adam(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                          const float* anchor, float* comm, const FLState* st, int local_step, hipStream_t s,
                          const MLPDescB* e, FLState* st_out, int fold, int tail_a, int fold_mask,
                          const PeerArgs* peer, int wx, int afold) {
    if (fold && st_out == nullptr) return hipErrorInvalidValue;
    // the exchanges' call index advances in the folded state: an exchange needs the fold
    if ((wx || afold) &&
        (peer == nullptr || !fold || local_step != c.local_steps - 1 || peer->n_chunks < (d.P + 63) / 64 + 2 ||
         (afold && (!tail_a || c.lag_off <= 0))))
        return hipErrorInvalidValue;
    PeerArgs pa;
    PeerArgs zero_pa = {};
    pa = zero_pa;
    if (peer != nullptr) pa = *peer;
    const int blocks = (d.P + 63) / 64 + 1;
    MLPDescB ee = {};
    if (e != nullptr) ee = *e;
#ifndef FL_ADAM_GENERAL_ONLY  // (A/B builds: every round through the general kernel)
    if (peer == nullptr && !wx && !afold)
        return fl_launch_adam_local(d, c, b, pin, anchor, comm, st, local_step, ee, e != nullptr ? 1 : 0, st_out, fold,
                                    tail_a, fold_mask, s);
    if (pa.ll != nullptr)
        return fl_launch_adam_ll(d, c, b, pin, anchor, comm, st, local_step, ee, e != nullptr ? 1 : 0, st_out, fold,
                                 tail_a, fold_mask, pa, wx ? 1 : 0, afold ? 1 : 0, s);
#endif
    if ((wx || afold) && pa.adam_grid > 0 && pa.adam_grid < blocks) {
        hipLaunchKernelGGL(fl_adam_grid_kernel, dim3(pa.adam_grid), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin, anchor,
                           comm, st, local_step, ee, e != nullptr ? 1 : 0, st_out, fold, tail_a, fold_mask, pa,
                           wx ? 1 : 0, afold ? 1 : 0, blocks);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(fl_adam_kernel, dim3(blocks), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin, anchor, comm, st,
                       local_step, ee, e != nullptr ? 1 : 0, st_out, fold, tail_a, fold_mask, pa, wx ? 1 : 0,
                       afold ? 1 : 0);
    return hipGetLastError();
}

template <int RT>
static hipError_t launch_eval_rt(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* params,
                                 float* cm, const FLState* st, hipStream_t s) {
    hipLaunchKernelGGL(fl_eval_kernel<RT>, dim3(nblocks(c.n_rows, RT * 16)), dim3(FL_THREADS), lds_bytes(d), s, d,
                       c, b, params, cm, st);
    return hipGetLastError();
}

hipError_t fl_launch_eval(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* params,
                          float* comm, const FLState* st, hipStream_t s) {
    float* cm = comm + c.tail_off + c.rank * c.tail_stride;
    switch (c.R) {
        case 16: return launch_eval_rt<1>(d, c, b, params, cm, st, s);
        case 32: return launch_eval_rt<2>(d, c, b, params, cm, st, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t fl_launch_eval_fedavg(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* params,
                                 float* comm, const FLState* st, const PeerArgs& a, const PeerPack& pk,
                                 hipStream_t s) {
    float* cm = comm + c.tail_off + c.rank * c.tail_stride;
    const int blocks = nblocks(c.n_rows, c.R);
    const int n_ar = fl_fedavg_blocks(a.n_w);
    if (a.eflags == nullptr || a.n_eval != blocks) return hipErrorInvalidValue;
    switch (c.R) {
        case 16:
            hipLaunchKernelGGL(fl_eval_fedavg_kernel<1>, dim3(n_ar + blocks), dim3(FL_THREADS), lds_bytes(d), s, d, c,
                               b, params, cm, st, a, pk, n_ar);
            break;
        case 32:
            hipLaunchKernelGGL(fl_eval_fedavg_kernel<2>, dim3(n_ar + blocks), dim3(FL_THREADS), lds_bytes(d), s, d, c,
                               b, params, cm, st, a, pk, n_ar);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_finalize(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, float* pg,
                              const FLState* si, FLState* so, hipStream_t s, int mask, const float* prev_out) {
    if ((d.Pimg & 3) != 0) return hipErrorInvalidValue;  // the image copy moves float4s
    hipLaunchKernelGGL(fl_finalize_kernel, dim3(1), dim3(64), 0, s, d, c, b, pg, si, so, mask, prev_out);
    return hipGetLastError();
}

hipError_t fl_launch_train_batch(const MLPDesc& d, int R, int n_slabs, const FLTrialDesc* T, int K, FLSel pg,
                                 FLSel si, FLSel so, int ls, int mode, FLSel cm, int fold_mask, hipStream_t s) {
    if (K < 1 || mode == FL_EVAL_LAGGED || (mode == FL_EVAL_FUSED && cm.base < 0)) return hipErrorInvalidValue;
    const dim3 grid(n_slabs, K);
    switch (R) {
        case 16:
            hipLaunchKernelGGL(fl_train_batch_kernel<1>, grid, dim3(FL_THREADS), lds_bytes(d), s, d, T, pg, si, so,
                               ls, mode, cm, fold_mask);
            break;
        case 32:
            hipLaunchKernelGGL(fl_train_batch_kernel<2>, grid, dim3(FL_THREADS), lds_bytes(d), s, d, T, pg, si, so,
                               ls, mode, cm, fold_mask);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_eval_batch(const MLPDesc& d, int R, int n_rows, const FLTrialDesc* T, int K, FLSel params,
                                FLSel comm, FLSel st, hipStream_t s) {
    if (K < 1) return hipErrorInvalidValue;
    const dim3 grid(nblocks(n_rows, R), K);
    switch (R) {
        case 16:
            hipLaunchKernelGGL(fl_eval_batch_kernel<1>, grid, dim3(FL_THREADS), lds_bytes(d), s, d, T, params, comm,
                               st);
            break;
        case 32:
            hipLaunchKernelGGL(fl_eval_batch_kernel<2>, grid, dim3(FL_THREADS), lds_bytes(d), s, d, T, params, comm,
                               st);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_finalize_batch(const MLPDesc& d, const FLTrialDesc* T, int K, FLSel pg, FLSel si, FLSel so,
                                    int mask, hipStream_t s) {
    if (K < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fl_finalize_batch_kernel, dim3(1, K), dim3(64), 0, s, d, T, pg, si, so, mask);
    return hipGetLastError();
}

hipError_t fl_launch_confusion(const MLPDesc& d, int R, const float* X, const int* y, int n_rows,
                               const float* params, float* cm_out, hipStream_t s) {
    FLConfig c = {};
    c.R = R;
    c.n_rows = n_rows;
    FLBuffers b = {};
    b.X = X;
    b.y = y;
    switch (R) {
        case 16: return launch_eval_rt<1>(d, c, b, params, cm_out, nullptr, s);
        case 32: return launch_eval_rt<2>(d, c, b, params, cm_out, nullptr, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t fl_launch_synth(float* X, int* y, long long n, int F, unsigned long long seed,
                           unsigned long long row_offset, const float* w1, const float* w2, int H,
                           hipStream_t s, float label_noise) {
    if (F > 32) return hipErrorInvalidValue;
    const long long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(fl_synth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X, y, n, F, seed, row_offset,
                       w1, w2, H, label_noise);
    return hipGetLastError();
}

// One wave that sleeps for `ticks` of the 100 MHz s_memrealtime clock: holds a stream while
// the host enqueues an eagerly traced sequence behind it (FLEngine::trace), so the traced
// kernels run back to back instead of at the host's launch pace.  Bounded: it always exits.
__global__ void fl_gate_kernel(long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(64);
}

hipError_t fl_launch_gate(double us, hipStream_t s) {
    if (!(us >= 0.0) || us > 1e6) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fl_gate_kernel, dim3(1), dim3(64), 0, s, (long long)(us * 100.0));
    return hipGetLastError();
}

// Allow the LDS-resident kernels to request more than the default dynamic-LDS window
// (gfx950 has 160 KiB per CU).
hipError_t fl_set_lds_limit(size_t bytes) {
    const int b = (int)bytes;
    hipError_t e = hipSuccess;
#define FL_SET(fn)                                                                                      \
    if (e == hipSuccess)                                                                                \
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, b)
    FL_SET(fl_train_kernel<1>); FL_SET(fl_train_kernel<2>);
    FL_SET(fl_train_batch_kernel<1>); FL_SET(fl_train_batch_kernel<2>);
    FL_SET(fl_eval_kernel<1>); FL_SET(fl_eval_kernel<2>);
    FL_SET(fl_eval_batch_kernel<1>); FL_SET(fl_eval_batch_kernel<2>);
    FL_SET(fl_eval_fedavg_kernel<1>); FL_SET(fl_eval_fedavg_kernel<2>);
#undef FL_SET
    return e;
}
