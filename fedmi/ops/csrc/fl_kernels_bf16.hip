// bf16-operand fused round kernels for gfx950 (BASELINE config 2: "3-layer MLP bf16").
//
// Same round structure, state machine, slab and Adam kernel as the fp32 path
// (fl_kernels.hip); only the per-workgroup GEMM work changes:
//
//   * the fp32 parameter image (global, all-reduced in fp32) is kept pre-packed as a bf16 LDS
//     image (hi parts, fp32 biases, lo parts); activations and deltas live in LDS as bf16,
//     accumulation is fp32 and the weight gradients written to the slab are fp32 (fp32 master
//     weights + Adam state);
//   * the forward pass is split-bf16 (fl_common.h): a_hi.W_hi + a_lo.W_hi + a_hi.W_lo, so the
//     logits that score the model (and drive the early-stop rule) carry ~16 significant bits;
//     the backward pass multiplies the hi parts only;
//   * all GEMMs run on v_mfma_f32_16x16x32_bf16 (16x the fp32 MFMA rate per FLOP):
//       fwd    z  = act . W^T      A = act rows (ds_read_b128), B = W rows (ds_read_b128)
//       dgrad  D  = D' . W         A = D' rows (ds_read_b128), B = W^T  via ds_read_b64_tr_b16
//       wgrad  dW = D'^T . act     A = D'^T, B = act^T, both via ds_read_b64_tr_b16 (K = rows)
//     so no transposed copy of any operand is ever stored: the hardware transpose read
//     serves the column-wise uses of the same row-major images;
//   * with R = 16 rows per workgroup the row contraction of wgrad is 16 deep and uses
//     v_mfma_f32_16x16x16_bf16 (one transposed read per operand).
//
// Reference semantics: forward/backward of MLPModel + CrossEntropyLoss
// (FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:12-25, 63-73), evaluation C:75-91.
#include "fl_common.h"
#include "fl_device.h"
#include "peer_device.h"
#include <math.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4* lds_bf16x4_ptr;

// fp32 -> bf16 bits, round to nearest even (finite inputs)
__device__ __forceinline__ uint32_t bf16_bits(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) { return bf16_bits(a) | (bf16_bits(b) << 16); }
// lo parts of the split-bf16 representation: bf16(x - bf16(x))
__device__ __forceinline__ uint32_t lo_bits(float x) { return bf16_bits(x - bf16_to_f32((uint16_t)bf16_bits(x))); }
__device__ __forceinline__ uint32_t pack_lo_bf16x2(float a, float b) { return lo_bits(a) | (lo_bits(b) << 16); }

// two fp32 -> packed bf16 pair (a low, b high), round to nearest even: v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    const bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ bf16x8 ld128(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group passes &M[r0+q][c0+4p]; lane i of the
// group receives M[r0+0..3][c0+i].
__device__ __forceinline__ bf16x4 ld_tr(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_ptr)(p));
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
    return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------
// Staging
// ---------------------------------------------------------------------------------------
// fp32 global image (fl_common.h layout) -> packed bf16 parameter region (MLPDescB layout,
// W_l then b_l, byte offsets relative to param_off).  One thread per 8-element item (two
// float4 loads, one 16-byte store); rows/columns of padding come out zero.
__device__ __forceinline__ void fl_pack_bf16_body(const MLPDesc& d, const MLPDescB& e, const float* __restrict__ params,
                                                  char* __restrict__ out) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = e.item_base[d.L];
    if (id < total) {
        int l = 0;
#pragma unroll
        for (int q = 1; q < FL_MAX_LAYERS; ++q) l += (q < d.L && id >= e.item_base[q]) ? 1 : 0;
        const int loc = id - e.item_base[l];
        const int nch = e.kp[l] >> 3;
        const int n = loc / nch, ch = loc - n * nch;
        const int K16 = (d.dim[l] + 15) & ~15, N16 = (d.dim[l + 1] + 15) & ~15;
        const bool ok = n < N16 && 8 * ch < K16;
        uint4 v = make_uint4(0u, 0u, 0u, 0u), w = make_uint4(0u, 0u, 0u, 0u);
        if (ok) {
            const float4* src = reinterpret_cast<const float4*>(params + d.iw_off[l] + n * fl_ldw(d.dim[l]) + 8 * ch);
            const bool sw = fl_swz(n) != 0;  // the image's swizzled rows hold the two halves swapped
            const float4 p0 = sw ? src[1] : src[0], p1 = sw ? src[0] : src[1];
            v = make_uint4(pack_bf16x2(p0.x, p0.y), pack_bf16x2(p0.z, p0.w), pack_bf16x2(p1.x, p1.y),
                           pack_bf16x2(p1.z, p1.w));
            w = make_uint4(pack_lo_bf16x2(p0.x, p0.y), pack_lo_bf16x2(p0.z, p0.w), pack_lo_bf16x2(p1.x, p1.y),
                           pack_lo_bf16x2(p1.z, p1.w));
        }
        char* dst = out + e.w_off[l] - e.param_off + fl_wrow(n, e.ldw[l], e.wgap) + 16 * (ch ^ fl_wswz(n, e.wxor));
        *reinterpret_cast<uint4*>(dst) = v;
        *reinterpret_cast<uint4*>(dst + e.wlo_delta) = w;
        return;
    }
    int bid = id - total;
    for (int l = 0; l < d.L; ++l) {
        if (bid < e.kp[l + 1]) {
            const int N16 = (d.dim[l + 1] + 15) & ~15;
            reinterpret_cast<float*>(out + e.bias_off[l] - e.param_off)[bid] = bid < N16 ? params[d.ib_off[l] + bid] : 0.f;
            return;
        }
        bid -= e.kp[l + 1];
    }
}

__global__ void fl_pack_bf16_kernel(MLPDesc d, MLPDescB e, const float* __restrict__ params, char* __restrict__ out) {
    fl_pack_bf16_body(d, e, params, out);
}

__global__ void fl_pack_bf16_batch_kernel(MLPDesc d, MLPDescB e, const FLTrialDesc* __restrict__ T, FLSel params,
                                          FLSel out) {
    const FLTrialDesc& t = T[blockIdx.y];
    fl_pack_bf16_body(d, e, reinterpret_cast<const float*>(fl_sel(t, params)), fl_sel(t, out));
}

// Stage the packed parameter region AND this block's input rows with every global load in
// flight before the first LDS store: the two ~1 us L2 latencies overlap instead of adding.
// Loads beyond STAGE_UNROLL per thread (large models) fall back to a loop.  The rows go to LDS
// split: act_0 = bf16(x), alo_0 = bf16(x - bf16(x)).
#define STAGE_P_UNROLL 8
#define STAGE_X_UNROLL 2
// NT: the staging threads (threads [0, NT); lagged rounds scored in registers leave the scoring
// waves out, fwd_sync).
// PLAIN (plain-bf16 training forward, FLConfig::plain_fwd): only the hi images and the biases
// (the region's first w_off[0] + wlo_delta bytes) are staged -- half the bytes.
template <int RT, int NT = FL_THREADS, bool PLAIN = false>
__device__ __forceinline__ void stage_params_rows_bf16(const MLPDescB& e, const char* __restrict__ packed,
                                                       const float* __restrict__ X, int n_rows, int F, int row0,
                                                       char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    uint4* dst = reinterpret_cast<uint4*>(lds + e.param_off);
    const int n16 = (PLAIN ? e.w_off[0] - e.param_off + e.wlo_delta : e.param_bytes) >> 4;
    const int kp = e.kp[0], lda = e.lda[0];
    const int nx = RT * 16 * kp;
    float xv[STAGE_X_UNROLL];
#ifndef FL_STAGE_VGPR
    // the parameter region goes global -> LDS by DMA (global_load_lds_dwordx4: 1 KB per wave
    // instruction, no VGPR round trip, no ds_write), the rows' loads issued first; the region's
    // last partial 1 KB is exec-masked (the head partials follow it in LDS)
#pragma unroll
    for (int u = 0; u < STAGE_X_UNROLL; ++u) {
        const int idx = threadIdx.x + u * NT;
        const int r = idx / kp, k = idx - r * kp;
        const int row = row0 + r;
        const bool ok = idx < nx && row < n_rows && k < F && (NT == FL_THREADS || (int)threadIdx.x < NT);
        const float v = X[ok ? (size_t)row * F + k : 0];
        xv[u] = ok ? v : 0.f;
    }
    {
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        for (int c0 = wv * 64; c0 < n16 && (NT == FL_THREADS || wv < NT / 64); c0 += NT)
            if (c0 + ln < n16)
                __builtin_amdgcn_global_load_lds(packed + (size_t)(c0 + ln) * 16,
                                                 (__attribute__((address_space(3))) void*)(lds + e.param_off + c0 * 16),
                                                 16, 0, 0);
    }
#else
    static_assert(NT == FL_THREADS && !PLAIN, "FL_STAGE_VGPR stages the whole region with every thread");
    uint4 pv[STAGE_P_UNROLL];
    // unpredicated loads (clamped indices): a conditionally written register array is
    // demoted to scratch by the compiler
#pragma unroll
    for (int u = 0; u < STAGE_P_UNROLL; ++u) {
        const int i = threadIdx.x + u * FL_THREADS;
        pv[u] = src[i < n16 ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < STAGE_X_UNROLL; ++u) {
        const int idx = threadIdx.x + u * NT;
        const int r = idx / kp, k = idx - r * kp;
        const int row = row0 + r;
        const bool ok = idx < nx && row < n_rows && k < F && (NT == FL_THREADS || (int)threadIdx.x < NT);
        const float v = X[ok ? (size_t)row * F + k : 0];
        xv[u] = ok ? v : 0.f;
    }
    // pin every load here (an empty asm consuming the registers): otherwise the compiler
    // sinks each load into its conditional store below and the latencies serialise again
#pragma unroll
    for (int u = 0; u < STAGE_P_UNROLL; ++u) asm volatile("" ::"v"(pv[u].x), "v"(pv[u].y), "v"(pv[u].z), "v"(pv[u].w));
#pragma unroll
    for (int u = 0; u < STAGE_X_UNROLL; ++u) asm volatile("" ::"v"(xv[u]));
    for (int i = threadIdx.x + STAGE_P_UNROLL * FL_THREADS; i < n16; i += FL_THREADS) dst[i] = src[i];
#pragma unroll
    for (int u = 0; u < STAGE_P_UNROLL; ++u) {
        const int i = threadIdx.x + u * FL_THREADS;
        if (i < n16) dst[i] = pv[u];
    }
#endif
    uint16_t* a = reinterpret_cast<uint16_t*>(lds + e.act_off[0]);
    uint16_t* alo = reinterpret_cast<uint16_t*>(lds + e.alo_off[0]);
#pragma unroll
    for (int u = 0; u < STAGE_X_UNROLL; ++u) {
        const int idx = threadIdx.x + u * NT;
        if (idx < nx && (NT == FL_THREADS || (int)threadIdx.x < NT)) {
            const int r = idx / kp, k = idx - r * kp;
            a[r * lda + k] = (uint16_t)bf16_bits(xv[u]);
            alo[r * lda + k] = (uint16_t)lo_bits(xv[u]);
        }
    }
    for (int idx = threadIdx.x + STAGE_X_UNROLL * NT; idx < nx && (NT == FL_THREADS || (int)threadIdx.x < NT);
         idx += NT) {
        const int r = idx / kp, k = idx - r * kp;
        const int row = row0 + r;
        const bool ok = row < n_rows && k < F;
        const float v = ok ? X[(size_t)row * F + k] : 0.f;
        a[r * lda + k] = (uint16_t)bf16_bits(v);
        alo[r * lda + k] = (uint16_t)lo_bits(v);
    }
#ifndef FL_STAGE_VGPR
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA has written the region (barrier follows)
#endif
}

// Register half of a parameter-region copy (FL_EVAL_LAGGED: the round's own weights are
// loaded while the previous local model is scored, and stored once that pass is done).
struct ParamRegs {
    uint4 v[STAGE_P_UNROLL];
};
__device__ __forceinline__ void params_load(const MLPDescB& e, const char* __restrict__ packed, ParamRegs& pr) {
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    const int n16 = e.param_bytes >> 4;
#pragma unroll
    for (int u = 0; u < STAGE_P_UNROLL; ++u) {
        const int i = threadIdx.x + u * FL_THREADS;
        pr.v[u] = src[i < n16 ? i : 0];
    }
}
__device__ __forceinline__ void params_store(const MLPDescB& e, const char* __restrict__ packed, const ParamRegs& pr,
                                             char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    uint4* dst = reinterpret_cast<uint4*>(lds + e.param_off);
    const int n16 = e.param_bytes >> 4;
#pragma unroll
    for (int u = 0; u < STAGE_P_UNROLL; ++u) {
        const int i = threadIdx.x + u * FL_THREADS;
        const uint4 v = pr.v[u];
        if (i < n16) dst[i] = v;
    }
    for (int i = threadIdx.x + STAGE_P_UNROLL * FL_THREADS; i < n16; i += FL_THREADS) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------
// GEMM phases (operand maps of v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4)+j]
// and B[8(l>>4)+j][l&15]; C/D col l&15, row 4(l>>4)+j)
// ---------------------------------------------------------------------------------------

// z = act_l . W_l^T + b_l in split bf16 (fl_common.h): hi.hi in `acc`, the two cross terms in
// `acl` (independent accumulation chains), z = acc + acl.  Hidden layers: ReLU -> act_{l+1}
// hi / lo parts (all kp[l+1] columns, the padding comes out 0); last layer: fp32 logits [R][16].
// NWV: waves that take the tiles (FL_WAVES; lagged rounds scored in registers: the first
// FL_WAVES - FL_LAG_SPR RT, fwd_sync).
// PLAIN: a_hi.W_hi only (the training forward of several clients, FLConfig::plain_fwd): no lo
// operands, no lo parts of the outputs.
template <int RT, int NWV = FL_WAVES, bool PLAIN = false>
__device__ __forceinline__ void fwd_layer_bf16(const MLPDesc& d, const MLPDescB& e, int l, char* lds) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    const bool last = (l + 1 == d.L);
    const int ntiles = last ? ((d.dim[d.L] + 15) >> 4) : (e.kp[l + 1] >> 4);
    const int ksteps = e.kp[l] >> 5;
    const int lda = e.lda[l];
    const char* W = lds + e.w_off[l];
    const char* act = lds + e.act_off[l];
    const char* alo = lds + e.alo_off[l];
    const float* bias = reinterpret_cast<const float*>(lds + e.bias_off[l]);
    const int wc = fl_fwd_col(lr);  // this lane's W row / output column within the tile
    const int wlane = 16 * (lg ^ fl_wswz(wc, e.wxor));  // its chunk of each k-step (swizzled)
    for (int nt = wave; nt < ntiles; nt += NWV) {
        if (NWV < FL_WAVES && wave >= NWV) break;
        const char* wrow = W + fl_wrow(nt * 16 + wc, e.ldw[l], e.wgap) + wlane;
        const int aoff = (lr * lda + 8 * lg) * 2;
        f32x4 acc[RT], acl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            acc[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
            acl[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        for (int ks = 0; ks < ksteps; ++ks) {
            const bf16x8 bv = ld128(wrow + ks * 64);
            if constexpr (PLAIN) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(ld128(act + aoff + rt * 16 * lda * 2 + ks * 64), bv, acc[rt]);
                continue;
            }
            const bf16x8 bl = ld128(wrow + e.wlo_delta + ks * 64);
            bf16x8 av[RT], al[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                av[rt] = ld128(act + aoff + rt * 16 * lda * 2 + ks * 64);
                al[rt] = ld128(alo + aoff + rt * 16 * lda * 2 + ks * 64);
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                acc[rt] = mfma32(av[rt], bv, acc[rt]);
                acl[rt] = mfma32(al[rt], bv, acl[rt]);
                acl[rt] = mfma32(av[rt], bl, acl[rt]);
            }
        }
        const int n = nt * 16 + wc;
        const float b = bias[n];
        const bool odd = lg & 1;
        if (last) {
            float* z = reinterpret_cast<float*>(lds + e.logit_off);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float v = odd ? acc[rt][(t + 1) & 3] + acl[rt][(t + 1) & 3] : acc[rt][t] + acl[rt][t];
                    z[(rt * 16 + fl_out_row(lg, t)) * FL_LOGIT_LD + n] = v + b;
                }
        } else {
            uint16_t* out = reinterpret_cast<uint16_t*>(lds + e.act_off[l + 1]);
            uint16_t* olo = reinterpret_cast<uint16_t*>(lds + e.alo_off[l + 1]);
            const int ldo = e.lda[l + 1];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int t = 0; t < 4; t += 2) {
                    if constexpr (NWV == FL_WAVES && !PLAIN) {  // the one-client kernel: software rounding
                        // (the same bits; the hardware form below measured +1.3 us on its round)
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const int u = t + q;
                            const float z = odd ? acc[rt][(u + 1) & 3] + acl[rt][(u + 1) & 3] : acc[rt][u] + acl[rt][u];
                            const float v = fmaxf(z + b, 0.f);
                            const int o = (rt * 16 + fl_out_row(lg, u)) * ldo + n;
                            out[o] = (uint16_t)bf16_bits(v);
                            olo[o] = (uint16_t)lo_bits(v);
                        }
                        continue;
                    }
                    // two rows per hi / lo conversion (v_cvt_pk_bf16_f32: bf16_bits / lo_bits' bits)
                    float v[2];
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const int u = t + q;
                        const float z = odd ? acc[rt][(u + 1) & 3] + acl[rt][(u + 1) & 3] : acc[rt][u] + acl[rt][u];
                        v[q] = fmaxf(z + b, 0.f);
                    }
                    const uint32_t h = cvt_pk_bf16(v[0], v[1]);
                    const int o0 = (rt * 16 + fl_out_row(lg, t)) * ldo + n, o1 = (rt * 16 + fl_out_row(lg, t + 1)) * ldo + n;
                    out[o0] = (uint16_t)h;
                    out[o1] = (uint16_t)(h >> 16);
                    if constexpr (!PLAIN) {
                        const uint32_t lo =
                            cvt_pk_bf16(v[0] - __uint_as_float(h << 16), v[1] - __uint_as_float(h & 0xffff0000u));
                        olo[o0] = (uint16_t)lo;
                        olo[o1] = (uint16_t)(lo >> 16);
                    }
                }
        }
    }
}

// dW_l[o][i] = sum_r D_{l+1}[r][o] act_l[r][i] (fp32 accumulate -> slab, dense [N][K]);
// gb_l[o] = sum_r D_{l+1}[r][o].  Both operands are read transposed (K = rows).  F16: the slab
// holds fp16 partials (element e at half e of the row, fl_device.h slab_store_h), else fp32.
template <bool F16>
__device__ __forceinline__ void slab_put(float* slab, int idx, float v) {
    if (F16) slab_store_h(reinterpret_cast<uint16_t*>(slab) + idx, v);
    else slab_store(slab + idx, v);
}
// Tiles go to waves [0, nw).  nw < FL_WAVES (waves nw.. run a long dgrad, wgrad_waves_bf16):
// handed out from wave nw-1 down, so the low waves, which also sum the biases (threads 0..),
// get the fewest.  nw = FL_WAVES: from wave 0 up (the dgrad items pair with them from the top).
template <int RT, bool F16>
__device__ void wgrad_layer_bf16(const MLPDesc& d, const MLPDescB& e, int l, const char* lds, float* __restrict__ slab,
                                 int nw) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4, lq = lr >> 2, lp = lr & 3;
    const int K = d.dim[l], N = d.dim[l + 1];
    const int otiles = (N + 15) >> 4, itiles = (K + 15) >> 4;
    const int ldd = e.lda[l + 1], lda = e.lda[l];
    const char* D = lds + e.dlt_off[l + 1];
    const char* act = lds + e.act_off[l];
    const int t0 = nw == FL_WAVES ? wave : (wave < nw ? nw - 1 - wave : otiles * itiles);
    for (int t = t0; t < otiles * itiles; t += nw) {
        const int ot = t / itiles, it = t - ot * itiles;
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (RT >= 2) {  // 32-row K chunks; k-runs 4lg.. and 16+4lg.. (8 consecutive rows per read)
#pragma unroll
            for (int h = 0; h < RT / 2; ++h) {
                const int r0 = 32 * h + 4 * lg + lq;
                const char* pa = D + (r0 * ldd + ot * 16 + 4 * lp) * 2;
                const char* pb = act + (r0 * lda + it * 16 + 4 * lp) * 2;
                const bf16x8 a = cat8(ld_tr(pa), ld_tr(pa + 16 * ldd * 2));
                const bf16x8 b = cat8(ld_tr(pb), ld_tr(pb + 16 * lda * 2));
                acc = mfma32(a, b, acc);
            }
        } else {
            const int r0 = 4 * lg + lq;
            const bf16x4 a = ld_tr(D + (r0 * ldd + ot * 16 + 4 * lp) * 2);
            const bf16x4 b = ld_tr(act + (r0 * lda + it * 16 + 4 * lp) * 2);
            acc = mfma16(a, b, acc);
        }
        const int i = it * 16 + lr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o = ot * 16 + 4 * lg + j;
            if (i < K && o < N) slab_put<F16>(slab, d.w_off[l] + o * K + i, acc[j]);
        }
    }
    const uint16_t* Dh = reinterpret_cast<const uint16_t*>(D);
    for (int o = threadIdx.x; o < N; o += FL_THREADS) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int r = 0; r < RT * 16; r += 2) {
            s0 += bf16_to_f32(Dh[r * ldd + o]);
            s1 += bf16_to_f32(Dh[(r + 1) * ldd + o]);
        }
        slab_put<F16>(slab, d.b_off[l] + o, s0 + s1);
    }
}

// Waves that take wgrad tiles in the backward phase of layer l.  The dgrad items (one per 16
// output columns, handed out from the last wave down) are chains of kp[l+1]/32 dependent
// k-steps; when they are long (the 50 -> 200 layer: 4 items of 7 steps) their waves take no
// wgrad tiles, which otherwise stack on top of the chain and set the phase's length; with
// the LDS arrival count that replaces the phase's barrier (fl_train_bf16_body.inc) the
// (50, 200) layer's backward phase went 3.9 -> 3.1 us and the round 23.8 -> 23.3 us
// (tools/probes/stamps_fine.py, profiles/ab_backward_waves_r2.log).  Short chains (the head's 1 step)
// share the waves with the tiles as before.  Only the work-to-wave map changes: every tile
// and item computes the same values.
__device__ __forceinline__ int wgrad_waves_bf16(const MLPDescB& e, int l) {
    const int items = l > 0 ? (e.kp[l] >> 4) : 0;
    const int steps = e.kp[l + 1] >> 5;
    return (items > 0 && steps >= 4 && 2 * items <= FL_WAVES) ? FL_WAVES - items : FL_WAVES;
}

// D_l[r][i] = (sum_o D_{l+1}[r][o] W_l[o][i]) * (act_l[r][i] > 0), all kp[l] columns.
// B = W_l^T through transposed reads of the row-major W image.  Items from the last wave
// down (pairs with wgrad's tiles handed out from wave 0 up).
template <int RT, bool HWCVT = false>
__device__ void dgrad_layer_bf16(const MLPDesc& d, const MLPDescB& e, int l, char* lds) {
    const int wave = (FL_WAVES - 1) - (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4, lq = lr >> 2, lp = lr & 3;
    const int itiles = e.kp[l] >> 4;
    const int osteps = e.kp[l + 1] >> 5;
    const int ldd = e.lda[l + 1], lda = e.lda[l], ldw = e.ldw[l];
    const char* Dn = lds + e.dlt_off[l + 1];
    const char* W = lds + e.w_off[l];
    const uint16_t* act = reinterpret_cast<const uint16_t*>(lds + e.act_off[l]);
    uint16_t* out = reinterpret_cast<uint16_t*>(lds + e.dlt_off[l]);
    for (int it = wave; it < itiles; it += FL_WAVES) {
        f32x4 acc[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // W rows 8lg+lq (+4), columns it*16 + 4lp..: 16-byte chunk 2it + lp/2, swizzled
        const char* pw = W + fl_wrow(8 * lg + lq, ldw, e.wgap) + 32 * it + 16 * ((lp >> 1) ^ fl_wswz(8 * lg, e.wxor)) +
                         8 * (lp & 1);
        const char* pa = Dn + (lr * ldd + 8 * lg) * 2;
        for (int os = 0; os < osteps; ++os) {
            const char* pwk = pw + os * (64 * ldw + 4 * e.wgap);  // fl_wrow(32 os + r) - fl_wrow(r)
            const bf16x8 bv = cat8(ld_tr(pwk), ld_tr(pwk + 4 * ldw * 2));
            bf16x8 av[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) av[rt] = ld128(pa + rt * 16 * ldd * 2 + os * 64);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(av[rt], bv, acc[rt]);
        }
        const int i = it * 16 + lr;
        const bool odd = lg & 1;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int t = 0; t < 4; t += 2) {
                if constexpr (!HWCVT) {  // software rounding (see fwd_layer_bf16)
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const int u = t + q;
                        const float g = odd ? acc[rt][(u + 1) & 3] : acc[rt][u];
                        const int o = (rt * 16 + fl_out_row(lg, u)) * lda + i;
                        out[o] = act[o] != 0 && !(act[o] & 0x8000u) ? (uint16_t)bf16_bits(g) : (uint16_t)0;
                    }
                    continue;
                }
                const float g0 = odd ? acc[rt][(t + 1) & 3] : acc[rt][t];
                const float g1 = odd ? acc[rt][(t + 2) & 3] : acc[rt][t + 1];
                const uint32_t h = cvt_pk_bf16(g0, g1);  // two rows per conversion (bf16_bits' bits)
                const int o0 = (rt * 16 + fl_out_row(lg, t)) * lda + i, o1 = (rt * 16 + fl_out_row(lg, t + 1)) * lda + i;
                out[o0] = act[o0] != 0 && !(act[o0] & 0x8000u) ? (uint16_t)h : (uint16_t)0;
                out[o1] = act[o1] != 0 && !(act[o1] & 0x8000u) ? (uint16_t)(h >> 16) : (uint16_t)0;
            }
    }
}

// Logits layer with its K loop split over e.head_split waves: wave w < G computes the split-bf16
// product over k-steps [w*kper, (w+1)*kper) of the single 16-column tile and drops its C useful
// columns into part[w][row][c]; after a barrier, thread (row, c) sums the G partials in order
// and adds the bias.  (One wave's chain of kp/32 dependent steps was the longest forward phase.)
// Forward-phase barrier.  PART (lagged rounds scored in registers): only the first
// FL_WAVES - FL_LAG_SPR RT waves run the forward pass, so they meet through an LDS arrival count (`tgt`
// grows by their number per phase) while the last FL_LAG_SPR RT waves score (score_out).
template <int RT, bool PART>
__device__ __forceinline__ void fwd_sync(int* cnt, int& tgt) {
    if constexpr (PART) {
        tgt += FL_WAVES - FL_LAG_SPR * RT;
        lds_count_arrive(cnt);
        lds_count_wait(cnt, tgt);
    } else {
        lds_barrier();
    }
}

template <int RT, bool PART = false, bool PLAIN = false>
__device__ __forceinline__ void fwd_head_split_bf16(const MLPDesc& d, const MLPDescB& e, char* lds, int* cnt,
                                                    int& tgt) {
    const int l = d.L - 1, C = d.dim[d.L], G = e.head_split;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    const int ksteps = e.kp[l] >> 5, kper = (ksteps + G - 1) / G;
    const int lda = e.lda[l];
    float* part = reinterpret_cast<float*>(lds + e.part_off);
    const int wc = fl_fwd_col(lr);
    if (wave < G) {
        const char* wrow = lds + e.w_off[l] + fl_wrow(wc, e.ldw[l], e.wgap) + 16 * (lg ^ fl_wswz(wc, e.wxor));
        const char* act = lds + e.act_off[l];
        const char* alo = lds + e.alo_off[l];
        const int aoff = (lr * lda + 8 * lg) * 2;
        f32x4 acc[RT], acl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            acc[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
            acl[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        const int k0 = wave * kper, k1 = min(ksteps, k0 + kper);
        for (int ks = k0; ks < k1; ++ks) {
            const bf16x8 bv = ld128(wrow + ks * 64);
            if constexpr (PLAIN) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(ld128(act + aoff + rt * 16 * lda * 2 + ks * 64), bv, acc[rt]);
                continue;
            }
            const bf16x8 bl = ld128(wrow + e.wlo_delta + ks * 64);
            bf16x8 av[RT], al[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                av[rt] = ld128(act + aoff + rt * 16 * lda * 2 + ks * 64);
                al[rt] = ld128(alo + aoff + rt * 16 * lda * 2 + ks * 64);
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                acc[rt] = mfma32(av[rt], bv, acc[rt]);
                acl[rt] = mfma32(al[rt], bv, acl[rt]);
                acl[rt] = mfma32(av[rt], bl, acl[rt]);
            }
        }
        if (wc < C) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int j = 0; j < 4; ++j) part[(wave * RT * 16 + rt * 16 + 4 * lg + j) * C + wc] = acc[rt][j] + acl[rt][j];
        }
    }
    fwd_sync<RT, PART>(cnt, tgt);
    const float* bias = reinterpret_cast<const float*>(lds + e.bias_off[l]);
    float* z = reinterpret_cast<float*>(lds + e.logit_off);
    for (int i = threadIdx.x; i < RT * 16 * C; i += FL_THREADS) {
        const int row = i / C, c = i - row * C;
        float s = part[row * C + c];
        for (int w = 1; w < G; ++w) s += part[(w * RT * 16 + row) * C + c];
        z[row * FL_LOGIT_LD + c] = s + bias[c];
    }
}

template <int RT, bool PART = false, bool PLAIN = false>
__device__ __forceinline__ void forward_block_bf16(const MLPDesc& d, const MLPDescB& e, char* lds, unsigned long long* dbg,
                                                   int* cnt = nullptr) {
    int tgt = 0;
    for (int l = 0; l < d.L; ++l) {
#ifndef FL_LAG_STAMPS
        if (dbg != nullptr && threadIdx.x == 0) dbg[blockIdx.x * 16 + 10 + l] = __builtin_amdgcn_s_memrealtime();
#endif
        if (l + 1 == d.L && e.head_split > 1) fwd_head_split_bf16<RT, PART, PLAIN>(d, e, lds, cnt, tgt);
        else fwd_layer_bf16<RT, PART ? FL_WAVES - FL_LAG_SPR * RT : FL_WAVES, PLAIN>(d, e, l, lds);
        fwd_sync<RT, PART>(cnt, tgt);
    }
}

// ---------------------------------------------------------------------------------------
// Register-resident scoring pass (FL_EVAL_LAGGED, several clients; fl_layout.h fl_lag_reg_ok)
// ---------------------------------------------------------------------------------------
// One wave scores 16 rows with the previous round's local model read straight from its packed
// global image (b.pk_local, L2-resident: every workgroup reads the same ~105 KB), so the LDS
// parameter region keeps the round's own weights and the scoring runs on the waves the
// training forward pass leaves idle, beside it instead of before it.  The product is computed
// transposed, Z^T = W . H^T: A = 16 W rows (global), B = the rows' activations, and the
// accumulator of a 16-feature tile -- lane (r, g) holds features 4g..4g+3 of row r -- becomes
// the next layer's B operand (lane (r, g): features 8g..8g+7 of a 32-deep k-block) after two
// lane swaps per tile pair (pair_to_b).  Every product sits at the same k position of the same
// v_mfma_f32_16x16x32_bf16 as in fwd_layer_bf16 / fwd_head_split_bf16 (only the roles of the
// A and B operands are exchanged), the split-bf16 chains and the bias / ReLU / hi-lo rounding
// are the same, and the logits' K-split partials are summed in the same order: the logits,
// hence the argmax counts, equal the evaluation kernel's (tests/test_peer_allreduce.py compares
// lagged rounds with classic ones bitwise).
// Profiling builds only (-DFL_LAG_STAMPS, tools/stamps.py): a stamp of the last scoring wave
// taken once `dep` (a value of the stage being timed) is available.
__device__ __forceinline__ void lag_stamp(const FLBuffers& b, int slot, uint32_t dep, bool on) {
#ifdef FL_LAG_STAMPS
    const uint32_t sdep = __builtin_amdgcn_readfirstlane(dep);
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "s"(sdep));
    if (on && b.dbg != nullptr && (threadIdx.x & 63) == 0) b.dbg[blockIdx.x * 16 + slot] = t;
#endif
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct TileBits {  // one transposed tile after bias + ReLU: hi / lo bf16 pairs of features 4g..4g+3
    uint32_t h0, h1, l0, l1;
};

// W_l rows nt*16 + m, k-block ks (A operand of the transposed product), hi and lo images.
__device__ __forceinline__ void score_ldw(const MLPDescB& e, const char* __restrict__ pk, int l, int nt, int ks, int m,
                                          int g, bf16x8& wh, bf16x8& wl) {
    const int n = nt * 16 + m;
    const char* p = pk + (e.w_off[l] - e.param_off) + fl_wrow(n, e.ldw[l], e.wgap) + 16 * (g ^ fl_wswz(n, e.wxor)) +
                    ks * 64;
    wh = *reinterpret_cast<const bf16x8*>(p);
    wl = *reinterpret_cast<const bf16x8*>(p + e.wlo_delta);
}
__device__ __forceinline__ f32x4 score_ldb(const MLPDescB& e, const char* __restrict__ pk, int l, int nt, int g) {
    return *reinterpret_cast<const f32x4*>(pk + (e.bias_off[l] - e.param_off) + (nt * 16 + 4 * g) * 4);
}

// One hidden-layer tile: split-bf16 chains in fwd_layer_bf16's order, z + b, ReLU, hi / lo.
template <int KB>
__device__ __forceinline__ TileBits score_tile(const bf16x8 (&wh)[KB], const bf16x8 (&wl)[KB], const bf16x8 (&bh)[KB],
                                               const bf16x8 (&bl)[KB], int nkb, f32x4 bias) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f}, acl = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {  // nkb == KB (callers instantiate the exact count)
        acc = mfma32(wh[kb], bh[kb], acc);
        acl = mfma32(wh[kb], bl[kb], acl);
        acl = mfma32(wl[kb], bh[kb], acl);
    }
    float v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = fmaxf((acc[t] + acl[t]) + bias[t], 0.f);
    // hi / lo parts with the hardware round-to-nearest-even conversion (v_cvt_pk_bf16_f32: the
    // bits of bf16_bits / lo_bits for finite values, a quarter of their VALU work)
    const uint32_t h01 = cvt_pk_bf16(v[0], v[1]), h23 = cvt_pk_bf16(v[2], v[3]);
    return TileBits{h01, h23, cvt_pk_bf16(v[0] - __uint_as_float(h01 << 16), v[1] - __uint_as_float(h01 & 0xffff0000u)),
                    cvt_pk_bf16(v[2] - __uint_as_float(h23 << 16), v[3] - __uint_as_float(h23 & 0xffff0000u))};
}

// Tiles 2kb, 2kb+1 (lane groups a_g, b_g) -> B operand of k-block kb.  Lane group g needs
// features 8g..8g+7 of the block: a_{2g}, a_{2g+1} for g < 2, b_{2g-4}, b_{2g-3} after.
// permlane32_swap(x, y) swaps x's upper half with y's lower half: x = [a0 a1 b0 b1],
// y = [a2 a3 b2 b3]; permlane16_swap then swaps x's odd rows with y's even rows:
// x = [a0 a2 b0 b2] (first 4 features of each group's 8), y = [a1 a3 b1 b3] (last 4).
__device__ __forceinline__ void pair_to_b(const TileBits& a, const TileBits& b, bf16x8& bh, bf16x8& bl) {
    const uint32_t xa[4] = {a.h0, a.h1, a.l0, a.l1}, xb[4] = {b.h0, b.h1, b.l0, b.l1};
    uint32_t f[4], s[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const auto r1 = __builtin_amdgcn_permlane32_swap(xa[i], xb[i], false, false);
        const auto r2 = __builtin_amdgcn_permlane16_swap(r1[0], r1[1], false, false);
        f[i] = r2[0];
        s[i] = r2[1];
    }
    bh = __builtin_bit_cast(bf16x8, (u32x4){f[0], f[1], s[0], s[1]});
    bl = __builtin_bit_cast(bf16x8, (u32x4){f[2], f[3], s[2], s[3]});
}

// The last hidden layer l (input B operand bh/bl, nkb k-blocks) streamed into the logits
// layer: each tile pair is one k-block of the logits' product, accumulated in the K-split
// parts of fwd_head_split_bf16 (part w = k-blocks [w*kper, (w+1)*kper), z = ((p_0 + p_1) + ...)
// + b; head_split 1 = fwd_layer_bf16's single chain).  FL_LAG_SPR waves share a 16-row group: wave
// `sj` takes parts [fl_lag_w(G, sj), fl_lag_w(G, sj + 1)) and their k-blocks; the upper waves store
// their parts in `parts` (LDS, lane group 0 = classes 0..3) and count themselves in `ready`, wave
// 0 adds them to its own running sum in part order -- the same additions in the same order as one
// wave (or fwd_head_split_bf16's partial sum) -- and returns the logits of lane (r, g): classes
// 4g..4g+3 of row r (the upper waves return nothing useful).  W tiles and biases are prefetched
// one tile ahead.
template <int KB>
__device__ __forceinline__ f32x4 score_hidden_head(const MLPDesc& d, const MLPDescB& e, const char* __restrict__ pk,
                                                   int l, const bf16x8 (&bh)[KB], const bf16x8 (&bl)[KB], int nkb,
                                                   int m, int g, int sj, f32x4* parts, int* ready,
                                                   const FLBuffers& b, bool last) {
    const int lh = d.L - 1;
    const int ntiles = e.kp[l + 1] >> 4, ksteps = ntiles >> 1;
    const int G = e.head_split, kper = (ksteps + G - 1) / G;
    // this wave's logits parts [wA, wB) and their k-blocks [ks0, ks1)
    const int wA = fl_lag_w(G, sj), wB = fl_lag_w(G, sj + 1);
    const int ks0 = min(ksteps, kper * wA), ks1 = min(ksteps, kper * wB);
    f32x4* myparts = parts + (sj > 0 ? (sj - 1) * FL_LAG_PARTS * 16 : 0);
    // buffer loads: the per-lane part of every address (W row m of a tile, its swizzled chunk g,
    // the bias entries of lane group g) is fixed, the tile / k-block part scalar -- no address
    // arithmetic per load
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pk), (short)0,
                                                                      e.param_bytes, 0x00020000);
    const int vw = m * e.ldw[l] * 2 + (m >> 3) * e.wgap + 16 * (g ^ fl_wswz(m, e.wxor));
    const int vh = m * e.ldw[lh] * 2 + (m >> 3) * e.wgap + 16 * (g ^ fl_wswz(m, e.wxor));
    const int vb = 16 * g;
    const int sw0 = e.w_off[l] - e.param_off, tstride = 32 * e.ldw[l] + 2 * e.wgap;
    const int sh0 = e.w_off[lh] - e.param_off, sb0 = e.bias_off[l] - e.param_off;
    auto ldw_t = [&](int nt, int kb, bf16x8& wh, bf16x8& wl) {
        const int so = sw0 + nt * tstride + kb * 64;
        wh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vw, so, 0));
        wl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vw, so + e.wlo_delta, 0));
    };
    auto ldb_t = [&](int nt) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vb, sb0 + nt * 64, 0));
    };
    auto ldh = [&](int ks, bf16x8& wh, bf16x8& wl) {
        wh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vh, sh0 + ks * 64, 0));
        wl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vh, sh0 + ks * 64 + e.wlo_delta, 0));
    };
    // two register sets, tile 2p from A while tile 2p+1 loads into B and the reverse: no
    // register copy of an in-flight load (a copy makes the compiler drain every load first)
    bf16x8 ah[KB], al[KB], bh2[KB], bl2[KB];
    const int tA = min(2 * ks0, ntiles - 1);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) ldw_t(tA, kb, ah[kb], al[kb]);
    f32x4 abias = ldb_t(tA), bbias;
    bf16x8 hh, hl;
    ldh(min(ks0, ksteps - 1), hh, hl);
    const f32x4 hb = score_ldb(e, pk, lh, 0, g);
    const f32x4 zero = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 acc = zero, acl = zero, s = zero;
    int w = wA, kend = min(ksteps, (w + 1) * kper);
    for (int ks = ks0; ks < ks1; ++ks) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) ldw_t(2 * ks + 1, kb, bh2[kb], bl2[kb]);
        bbias = ldb_t(2 * ks + 1);
        const TileBits t0 = score_tile<KB>(ah, al, bh, bl, nkb, abias);
        int nx = min(2 * ks + 2, ntiles - 1);
        // set A reloads after tile 2ks consumed all of it (no register copy)
        asm volatile("" : "+s"(nx) : "v"(t0.h0), "v"(t0.h1), "v"(t0.l0), "v"(t0.l1));
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) ldw_t(nx, kb, ah[kb], al[kb]);
        abias = ldb_t(nx);
        const TileBits t1 = score_tile<KB>(bh2, bl2, bh, bl, nkb, bbias);
#ifdef FL_LAG_STAMPS
        if (ks == 1) lag_stamp(b, 12, t1.h0, last);
#endif
        bf16x8 xh, xl;
        pair_to_b(t0, t1, xh, xl);
        acc = mfma32(hh, xh, acc);
        acl = mfma32(hh, xl, acl);
        acl = mfma32(hl, xh, acl);
        if (ks + 1 < ks1) ldh(ks + 1, hh, hl);
        if (ks + 1 == kend) {  // part w complete
            const f32x4 p = acc + acl;
            if (sj == 0) s = (w == 0) ? p : s + p;
            else if (g == 0) myparts[(w - wA) * 16 + m] = p;
            acc = zero;
            acl = zero;
            ++w;
            kend = min(ksteps, (w + 1) * kper);
        }
    }
    // empty trailing parts (0 + 0), as fwd_head_split_bf16 sums them
    if (sj == 0) {
        for (; w < wB; ++w) s = s + (acc + acl);
        lds_count_wait(ready, FL_LAG_SPR - 1);
        for (int j = 1; j < FL_LAG_SPR; ++j)
            for (int u = fl_lag_w(G, j); u < fl_lag_w(G, j + 1); ++u)
                s = s + parts[((j - 1) * FL_LAG_PARTS + u - fl_lag_w(G, j)) * 16 + m];
    } else {
        for (; w < wB; ++w)
            if (g == 0) myparts[(w - wA) * 16 + m] = acc + acl;
        lds_count_arrive(ready);
    }
    return s + hb;
}

struct ScoreIn {
    bf16x8 h[2], l[2];
};
// The first hidden layer's weights (<= 4 tiles, hi / lo / bias), loaded by the scoring waves at the
// kernel start -- they stage nothing -- so they land while the other waves stage (issued after the
// staging barrier they came from beyond the L2 in ~2 us, every CU asking for the same lines at once).
struct ScorePre {
    bf16x8 w0h[4][1], w0l[4][1];
    f32x4 b0[4];
};
template <int RT>
__device__ __forceinline__ void score_prefetch(const MLPDesc& d, const MLPDescB& e, const FLBuffers& b, ScorePre& pre) {
    if (d.L != 3) return;
    const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
    const int nt0 = e.kp[1] >> 4;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int t = nt < nt0 ? nt : 0;
        score_ldw(e, b.pk_local, 0, t, 0, r, g, pre.w0h[nt][0], pre.w0l[nt][0]);
        pre.b0[nt] = score_ldb(e, b.pk_local, 0, t, g);
    }
}

// Input side of a scoring wave `sw` (2 per 16-row group; rows row0 + 16 (sw / 2) + (0..15)), after
// the staging barrier: the staged rows (act_0 / alo_0, the B operand of the transposed product),
// and with two hidden layers the first one (weights from score_prefetch; both waves of the group)
// -> `in` = the B operand of the last hidden layer.  (Tried: the rows from global
// memory and the first layer before the staging barrier, with or without a first touch of every
// line of the local image -- the loads queue behind the staging's and delay the barrier;
// profiles/lag_reg_ab_r3.log.)
template <int RT>
__device__ __forceinline__ void score_in_lds(const MLPDesc& d, const MLPDescB& e, const FLBuffers& b, const char* lds,
                                             int sw, const ScorePre& pre, ScoreIn& in) {
    const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
    const int swu = __builtin_amdgcn_readfirstlane(sw);
    const int xo = ((16 * (swu / FL_LAG_SPR) + r) * e.lda[0] + 8 * g) * 2;
    bf16x8 xh[1], xl[1];
    xh[0] = ld128(lds + e.act_off[0] + xo);
    xl[0] = ld128(lds + e.alo_off[0] + xo);
    if (d.L == 2) {
        in.h[0] = xh[0];
        in.l[0] = xl[0];
        return;
    }
    const int nt0 = e.kp[1] >> 4;
    TileBits t0[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
        if (nt < nt0) t0[nt] = score_tile<1>(pre.w0h[nt], pre.w0l[nt], xh, xl, 1, pre.b0[nt]);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
        if (2 * kb < nt0) pair_to_b(t0[2 * kb], t0[2 * kb + 1], in.h[kb], in.l[kb]);
    lag_stamp(b, 11, t0[0].h0, swu == 0);
}

// Output side, after the staging barrier: the last hidden layer + logits (score_hidden_head,
// the group's FL_LAG_SPR waves splitting it), argmax -> cm_s (LDS ints) by the group's wave 0;
// ysc = the label of row r (lane r + 16 g).
template <int RT>
__device__ void score_out(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b, int* cm_s,
                          int sw, int row0, int ysc, const ScoreIn& in, f32x4* parts, int* ready) {
    const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
    const int swu = __builtin_amdgcn_readfirstlane(sw);  // wave-uniform: scalar tile indices
    const int sj = swu % FL_LAG_SPR;  // this wave's share of its row group (0: sums and counts)
    const char* __restrict__ pk = b.pk_local;
    const int C = d.dim[d.L];
    const int row = row0 + 16 * (swu / FL_LAG_SPR) + r;
    const bool last = swu == 0;
    if (b.dbg != nullptr && lane == 0 && last) b.dbg[blockIdx.x * 16 + 13] = __builtin_amdgcn_s_memrealtime();
    f32x4 z;
    if (d.L == 2) {
        const bf16x8 xh[1] = {in.h[0]}, xl[1] = {in.l[0]};
        z = score_hidden_head<1>(d, e, pk, 0, xh, xl, 1, r, g, sj, parts, ready, b, last);
    } else {
        if ((e.kp[1] >> 5) == 2) {
            z = score_hidden_head<2>(d, e, pk, 1, in.h, in.l, 2, r, g, sj, parts, ready, b, last);
        } else {
            const bf16x8 xh[1] = {in.h[0]}, xl[1] = {in.l[0]};
            z = score_hidden_head<1>(d, e, pk, 1, xh, xl, 1, r, g, sj, parts, ready, b, last);
        }
    }
    // stamps (tools/stamps.py): 13 = the first scoring wave past the staging barrier, 14 = its logits done
    if (b.dbg != nullptr && lane == 0 && last) b.dbg[blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memrealtime();
    // argmax over the C <= 4 classes of row r (torch.max: first maximum): lane group 0
    int best = 0;
    float bv = z[0];
#pragma unroll
    for (int k = 1; k < FL_LAG_MAX_C; ++k)
        if (k < C && z[k] > bv) { bv = z[k]; best = k; }
    if (sj == 0 && g == 0 && row < c.n_rows) atomicAdd(&cm_s[ysc * C + best], 1);
}

// A workgroup of the lagged round's SCORING blocks (train kernel LAG 3, FLConfig::split_score):
// the previous local model is scored for the rows of training block blockIdx.x - n_slabs by the
// same FL_LAG_SPR RT register-scoring waves, with the same wave numbering, as in the LAG 2 kernel
// -- but on a workgroup of their own, so the training blocks keep all 16 waves (their training is
// the non-lagged round's, bit for bit) and small shards, whose train grid leaves most CUs idle,
// score on the idle CUs.  The other waves end at once (s_barrier counts the live ones).  Counts:
// cm_s (LDS) -> cm_out, as the lagged training block flushes them.
// (No stamps: the debug buffer holds n_slabs blocks' rows.)
template <int RT>
__device__ void score_block_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b_in,
                                 const FLState* __restrict__ st_in, float* __restrict__ cm_out, char* lds,
                                 f32x4* lag_parts, int* lag_ready) {
    const int wave = threadIdx.x >> 6;
    constexpr int SW0 = FL_WAVES - FL_LAG_SPR * RT;  // first scoring wave
    if (wave < SW0) return;
    FLBuffers b = b_in;
    b.dbg = nullptr;
    const int t = (int)threadIdx.x - SW0 * 64;
    constexpr int NS = FL_LAG_SPR * RT * 64;      // scoring threads
    const int R = RT * 16, row0 = ((int)blockIdx.x - c.n_slabs) * R;
    const int C = d.dim[d.L];
    int* cm_s = reinterpret_cast<int*>(lds + e.cm_off);
    if (t < RT) lag_ready[t] = 0;
    for (int i = t; i < C * C; i += NS) cm_s[i] = 0;
    ScorePre spre;
    score_prefetch<RT>(d, e, b, spre);
    const int sw = wave - SW0;
    const int ysc = b.y[min(row0 + 16 * (sw / FL_LAG_SPR) + (int)(threadIdx.x & 15), c.n_rows - 1)];
    // the rows as split bf16 (act_0 hi / alo_0 lo), exactly as stage_params_rows_bf16 writes them
    {
        const int kp = e.kp[0], lda = e.lda[0], F = d.dim[0];
        uint16_t* a = reinterpret_cast<uint16_t*>(lds + e.act_off[0]);
        uint16_t* alo = reinterpret_cast<uint16_t*>(lds + e.alo_off[0]);
        for (int idx = t; idx < R * kp; idx += NS) {
            const int r = idx / kp, k = idx - r * kp;
            const int row = row0 + r;
            const bool ok = row < c.n_rows && k < F;
            const float v = ok ? b.X[(size_t)row * F + k] : 0.f;
            a[r * lda + k] = (uint16_t)bf16_bits(v);
            alo[r * lda + k] = (uint16_t)lo_bits(v);
        }
    }
    const FLState S0 = *st_in;  // the round's tentative live decision, as the training blocks take it
    const bool live = !S0.stopped && S0.next_round < c.max_rounds;
    lds_barrier();
    if (!live) return;
    ScoreIn sin;
    score_in_lds<RT>(d, e, b, lds, sw, spre, sin);
    score_out<RT>(d, e, c, b, cm_s, sw, row0, ysc, sin,
                  lag_parts + (sw / FL_LAG_SPR) * (FL_LAG_SPR - 1) * FL_LAG_PARTS * 16, lag_ready + sw / FL_LAG_SPR);
    lds_barrier();
    for (int i = t; i < C * C; i += NS)
        if (cm_s[i]) atomicAdd(&cm_out[i], (float)cm_s[i]);
}

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------
// Kernel body shared by the single-engine and trial-batch entry points (fl_train_bf16_body.inc).
// LAG: the lagged scoring pass (FL_EVAL_LAGGED, several clients) is compiled in -- 1: before
// the training pass (its register copy of the round's weights: R = 32 126 VGPRs), 2: in
// registers on the last 2 RT waves (score_rows_regs, shapes of fl_lag_reg_ok); the other modes get
// an instantiation without it (R = 32: 90 VGPRs; R = 64 spill-free).
template <int RT, int LAG, bool PLAIN>
__global__ void __launch_bounds__(FL_THREADS)
fl_train_bf16_kernel(MLPDesc d, MLPDescB e, FLConfig c, FLBuffers b, const float* __restrict__ pg,
                     const FLState* __restrict__ st_in, FLState* __restrict__ st_out, int local_step,
                     int stage_local, int mode, float* __restrict__ cm_out, int fold_mask) {
#include "fl_train_bf16_body.inc"
}

template <int RT, bool PLAIN>
__global__ void __launch_bounds__(FL_THREADS)
fl_train_bf16_batch_kernel(MLPDesc d, MLPDescB e, const FLTrialDesc* __restrict__ T, FLSel pg_sel, FLSel si_sel,
                           FLSel so_sel, int local_step, int stage_local, int mode, FLSel cm_sel, int fold_mask) {
    constexpr int LAG = 0;  // trial batches never run lagged rounds
    const FLTrialDesc& t = T[blockIdx.y];
    const FLConfig c = t.c;
    const FLBuffers b = t.b;
    const float* __restrict__ pg = reinterpret_cast<const float*>(fl_sel(t, pg_sel));
    const FLState* __restrict__ st_in = reinterpret_cast<const FLState*>(fl_sel(t, si_sel));
    FLState* __restrict__ st_out = reinterpret_cast<FLState*>(fl_sel(t, so_sel));
    float* __restrict__ cm_out = reinterpret_cast<float*>(fl_sel(t, cm_sel));
#include "fl_train_bf16_body.inc"
}

// Local evaluation of one row block (rows [blk*R, blk*R + R)) of the post-step model:
// forward, argmax, confusion counts added to cm_out (exact: integer-valued fp32 < 2^24).
template <int RT>
__device__ void eval_rows_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                               const float* __restrict__ params, float* __restrict__ cm_out, int blk, char* lds) {
    __shared__ int cm_s[FL_MAX_CLASSES * FL_MAX_CLASSES];
    const int R = RT * 16;
    const int row0 = blk * R;
    const int C = d.dim[d.L];
    FL_STAMP(0);
    for (int i = threadIdx.x; i < C * C; i += FL_THREADS) cm_s[i] = 0;
    const int ylab = (threadIdx.x < R) ? b.y[min(row0 + (int)threadIdx.x, c.n_rows - 1)] : 0;
    stage_params_rows_bf16<RT>(e, params == b.local ? b.pk_local : b.pk_global, b.X, c.n_rows, d.dim[0], row0,
                               lds);
    FL_STAMP(8);
    FL_STAMP(9);
    lds_barrier();
    FL_STAMP(1);
    forward_block_bf16<RT>(d, e, lds, nullptr);
    FL_STAMP(2);
    if (threadIdx.x < R) {
        const int r = threadIdx.x, row = row0 + r;
        if (row < c.n_rows) {
            const float* zr = reinterpret_cast<const float*>(lds + e.logit_off) + r * FL_LOGIT_LD;
            int best = 0;
            float bv = zr[0];
            for (int k = 1; k < C; ++k)
                if (zr[k] > bv) { bv = zr[k]; best = k; }
            atomicAdd(&cm_s[ylab * C + best], 1);
        }
    }
    lds_barrier();
    for (int i = threadIdx.x; i < C * C; i += FL_THREADS)
        if (cm_s[i]) atomicAdd(&cm_out[i], (float)cm_s[i]);
    FL_STAMP(15);
}

template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_eval_bf16_kernel(MLPDesc d, MLPDescB e, FLConfig c, FLBuffers b, const float* __restrict__ params,
                    float* __restrict__ cm_out, const FLState* __restrict__ st) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    if (st != nullptr && !st->live) return;
    eval_rows_bf16<RT>(d, e, c, b, params, cm_out, blockIdx.x, lds);
}

template <int RT>
__global__ void __launch_bounds__(FL_THREADS)
fl_eval_bf16_batch_kernel(MLPDesc d, MLPDescB e, const FLTrialDesc* __restrict__ T, FLSel params, FLSel comm,
                          FLSel st) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const FLTrialDesc& t = T[blockIdx.y];
    const FLState* s = reinterpret_cast<const FLState*>(fl_sel(t, st));
    if (s != nullptr && !s->live) return;
    float* cm = reinterpret_cast<float*>(fl_sel(t, comm)) + t.c.tail_off + t.c.rank * t.c.tail_stride;
    eval_rows_bf16<RT>(d, e, t.c, t.b, reinterpret_cast<const float*>(fl_sel(t, params)), cm, blockIdx.x, lds);
}

// Local evaluation + FedAvg in one kernel (world > 1, one-shot xGMI all-reduce;
// peer_device.h).  Blocks [0, n_ar) all-reduce: they pull and sum the peers' weights as soon
// as every rank published them -- the weights were complete when the Adam kernel ended --
// and, once every rank's evaluation is done, the metric tails.  Blocks [n_ar, grid) evaluate
// the post-step local model on the shard into this rank's tail slot; the last of them
// publishes the tails.  The all-reduce's waiting and xGMI latency hide behind the
// evaluation instead of following it.
template <int RT>
__global__ void __launch_bounds__(FL_THREADS, 8)  // 8 waves/SIMD = two workgroups per CU: one resident wave of blocks
fl_eval_fedavg_bf16_kernel(MLPDesc d, MLPDescB e, FLConfig c, FLBuffers b, const float* __restrict__ params,
                           float* __restrict__ cm_out, const FLState* __restrict__ st, PeerArgs a, PeerPack pk,
                           int n_ar) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const unsigned target = peer_target(a);
    if ((int)blockIdx.x < n_ar) {
        peer_fused_reduce(a, pk, target, blockIdx.x, n_ar);
        peer_finish(a, target, n_ar);
    } else {
        if (st->live) eval_rows_bf16<RT>(d, e, c, b, params, cm_out, blockIdx.x - n_ar, lds);
        peer_eval_done(a, target, blockIdx.x - n_ar);
    }
}

// ---------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------
hipError_t fl_launch_train_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                                const float* pg, const FLState* si, FLState* so, int ls, hipStream_t s,
                                bool stage_local, int mode, float* cm_out, int fold_mask) {
    if ((mode == FL_EVAL_FUSED || mode == FL_EVAL_LAGGED) && cm_out == nullptr) return hipErrorInvalidValue;
    const size_t lds = (size_t)e.lds_bytes;
    const bool lag = mode == FL_EVAL_LAGGED;
    // split scoring (FLConfig::split_score): the lagged round's first local step scores on
    // n_slabs workgroups of their own, appended to the grid (LAG 3)
    const bool lreg = lag && e.lag_reg;
    const bool split = lreg && c.split_score && ls == 0;
    const int grid = split ? 2 * c.n_slabs : c.n_slabs;
#define FLB_TRAIN(RT_, LAG_, PL_)                                                                           \
    hipLaunchKernelGGL((fl_train_bf16_kernel<RT_, LAG_, PL_>), dim3(grid), dim3(FL_THREADS), lds, s, d, e, c, b, pg, \
                       si, so, ls, stage_local ? 1 : 0, mode, cm_out, fold_mask)
    switch (c.R) {
        // plain_fwd (FLConfig): the training forward of several clients with register scoring (R <= 32)
        case 16:
            if (split) { if (c.plain_fwd) FLB_TRAIN(1, 3, true); else FLB_TRAIN(1, 3, false); }
            else if (lreg) { if (c.plain_fwd) FLB_TRAIN(1, 2, true); else FLB_TRAIN(1, 2, false); }
            else if (lag) FLB_TRAIN(1, 1, false);
            else if (c.plain_fwd) FLB_TRAIN(1, 0, true);
            else FLB_TRAIN(1, 0, false);
            break;
        case 32:
            if (split) { if (c.plain_fwd) FLB_TRAIN(2, 3, true); else FLB_TRAIN(2, 3, false); }
            else if (lreg) { if (c.plain_fwd) FLB_TRAIN(2, 2, true); else FLB_TRAIN(2, 2, false); }
            else if (lag) FLB_TRAIN(2, 1, false);
            else if (c.plain_fwd) FLB_TRAIN(2, 0, true);
            else FLB_TRAIN(2, 0, false);
            break;
        case 64: if (lag) FLB_TRAIN(4, 1, false); else FLB_TRAIN(4, 0, false); break;
        default: return hipErrorInvalidValue;
    }
#undef FLB_TRAIN
    return hipGetLastError();
}

hipError_t fl_launch_eval_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                               const float* params, float* comm, const FLState* st, hipStream_t s) {
    float* cm = comm + c.tail_off + c.rank * c.tail_stride;
    const int blocks = (c.n_rows + c.R - 1) / c.R;
    switch (c.R) {
        case 16:
            hipLaunchKernelGGL(fl_eval_bf16_kernel<1>, dim3(blocks), dim3(FL_THREADS), e.lds_bytes, s, d, e, c, b,
                               params, cm, st);
            break;
        case 32:
            hipLaunchKernelGGL(fl_eval_bf16_kernel<2>, dim3(blocks), dim3(FL_THREADS), e.lds_bytes, s, d, e, c, b,
                               params, cm, st);
            break;
        case 64:
            hipLaunchKernelGGL(fl_eval_bf16_kernel<4>, dim3(blocks), dim3(FL_THREADS), e.lds_bytes, s, d, e, c, b,
                               params, cm, st);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_eval_fedavg_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                                      const float* params, float* comm, const FLState* st, const PeerArgs& a,
                                      const PeerPack& pk, hipStream_t s) {
    float* cm = comm + c.tail_off + c.rank * c.tail_stride;
    const int blocks = (c.n_rows + c.R - 1) / c.R;
    const int n_ar = fl_fedavg_blocks(a.n_w);
    if (a.eflags == nullptr || a.n_eval != blocks) return hipErrorInvalidValue;
    switch (c.R) {
        case 16:
            hipLaunchKernelGGL(fl_eval_fedavg_bf16_kernel<1>, dim3(n_ar + blocks), dim3(FL_THREADS), e.lds_bytes, s, d,
                               e, c, b, params, cm, st, a, pk, n_ar);
            break;
        case 32:
            hipLaunchKernelGGL(fl_eval_fedavg_bf16_kernel<2>, dim3(n_ar + blocks), dim3(FL_THREADS), e.lds_bytes, s, d,
                               e, c, b, params, cm, st, a, pk, n_ar);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_pack_bf16(const MLPDesc& d, const MLPDescB& e, const float* params, char* out, hipStream_t s) {
    int bias_items = 0;
    for (int l = 0; l < d.L; ++l) bias_items += e.kp[l + 1];
    const int n = e.item_base[d.L] + bias_items;
    hipLaunchKernelGGL(fl_pack_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d, e, params, out);
    return hipGetLastError();
}

hipError_t fl_launch_train_bf16_batch(const MLPDesc& d, const MLPDescB& e, int R, int n_slabs, const FLTrialDesc* T,
                                      int K, FLSel pg, FLSel si, FLSel so, int ls, int stage_local, int mode, FLSel cm,
                                      int fold_mask, hipStream_t s, int plain) {
    if (K < 1 || mode == FL_EVAL_LAGGED || (mode == FL_EVAL_FUSED && cm.base < 0)) return hipErrorInvalidValue;
    if (plain && (R == 64 || mode == FL_EVAL_FUSED)) return hipErrorInvalidValue;
    const size_t lds = (size_t)e.lds_bytes;
    const dim3 grid(n_slabs, K);
    switch (R) {
        case 16:
            if (plain) hipLaunchKernelGGL((fl_train_bf16_batch_kernel<1, true>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so,
                                          ls, stage_local, mode, cm, fold_mask);
            else hipLaunchKernelGGL((fl_train_bf16_batch_kernel<1, false>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so, ls,
                               stage_local, mode, cm, fold_mask);
            break;
        case 32:
            if (plain) hipLaunchKernelGGL((fl_train_bf16_batch_kernel<2, true>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so,
                                          ls, stage_local, mode, cm, fold_mask);
            else hipLaunchKernelGGL((fl_train_bf16_batch_kernel<2, false>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so, ls,
                               stage_local, mode, cm, fold_mask);
            break;
        case 64:
            if (plain) hipLaunchKernelGGL((fl_train_bf16_batch_kernel<4, true>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so,
                                          ls, stage_local, mode, cm, fold_mask);
            else hipLaunchKernelGGL((fl_train_bf16_batch_kernel<4, false>), grid, dim3(FL_THREADS), lds, s, d, e, T, pg, si, so, ls,
                               stage_local, mode, cm, fold_mask);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_eval_bf16_batch(const MLPDesc& d, const MLPDescB& e, int R, int n_rows, const FLTrialDesc* T,
                                     int K, FLSel params, FLSel comm, FLSel st, hipStream_t s) {
    if (K < 1) return hipErrorInvalidValue;
    const dim3 grid((n_rows + R - 1) / R, K);
    switch (R) {
        case 16:
            hipLaunchKernelGGL(fl_eval_bf16_batch_kernel<1>, grid, dim3(FL_THREADS), e.lds_bytes, s, d, e, T, params,
                               comm, st);
            break;
        case 32:
            hipLaunchKernelGGL(fl_eval_bf16_batch_kernel<2>, grid, dim3(FL_THREADS), e.lds_bytes, s, d, e, T, params,
                               comm, st);
            break;
        case 64:
            hipLaunchKernelGGL(fl_eval_bf16_batch_kernel<4>, grid, dim3(FL_THREADS), e.lds_bytes, s, d, e, T, params,
                               comm, st);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t fl_launch_pack_bf16_batch(const MLPDesc& d, const MLPDescB& e, const FLTrialDesc* T, int K, FLSel params,
                                     FLSel out, hipStream_t s) {
    if (K < 1) return hipErrorInvalidValue;
    int bias_items = 0;
    for (int l = 0; l < d.L; ++l) bias_items += e.kp[l + 1];
    const int n = e.item_base[d.L] + bias_items;
    hipLaunchKernelGGL(fl_pack_bf16_batch_kernel, dim3((n + 255) / 256, K), dim3(256), 0, s, d, e, T, params, out);
    return hipGetLastError();
}

hipError_t fl_set_lds_limit_bf16(size_t bytes) {
    const int v = (int)bytes;
    hipError_t r = hipSuccess;
#define FLB_SET(fn)                                                                                     \
    if (r == hipSuccess)                                                                                \
    r = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, v)
    FLB_SET((fl_train_bf16_kernel<1, 0, false>)); FLB_SET((fl_train_bf16_kernel<2, 0, false>));
    FLB_SET((fl_train_bf16_kernel<4, 0, false>));
    FLB_SET((fl_train_bf16_kernel<1, 1, false>)); FLB_SET((fl_train_bf16_kernel<2, 1, false>));
    FLB_SET((fl_train_bf16_kernel<4, 1, false>));
    FLB_SET((fl_train_bf16_kernel<1, 2, false>)); FLB_SET((fl_train_bf16_kernel<2, 2, false>));
    FLB_SET((fl_train_bf16_kernel<1, 2, true>)); FLB_SET((fl_train_bf16_kernel<2, 2, true>));
    FLB_SET((fl_train_bf16_kernel<1, 0, true>)); FLB_SET((fl_train_bf16_kernel<2, 0, true>));
    FLB_SET((fl_train_bf16_kernel<1, 3, false>)); FLB_SET((fl_train_bf16_kernel<2, 3, false>));
    FLB_SET((fl_train_bf16_kernel<1, 3, true>)); FLB_SET((fl_train_bf16_kernel<2, 3, true>));
    FLB_SET(fl_eval_bf16_kernel<1>); FLB_SET(fl_eval_bf16_kernel<2>); FLB_SET(fl_eval_bf16_kernel<4>);
    FLB_SET((fl_train_bf16_batch_kernel<1, false>)); FLB_SET((fl_train_bf16_batch_kernel<2, false>));
    FLB_SET((fl_train_bf16_batch_kernel<4, false>)); FLB_SET((fl_train_bf16_batch_kernel<1, true>));
    FLB_SET((fl_train_bf16_batch_kernel<2, true>)); FLB_SET((fl_train_bf16_batch_kernel<4, true>));
    FLB_SET(fl_eval_bf16_batch_kernel<1>); FLB_SET(fl_eval_bf16_batch_kernel<2>); FLB_SET(fl_eval_bf16_batch_kernel<4>);
    FLB_SET(fl_eval_fedavg_bf16_kernel<1>); FLB_SET(fl_eval_fedavg_bf16_kernel<2>);
#undef FLB_SET
    return r;
}
