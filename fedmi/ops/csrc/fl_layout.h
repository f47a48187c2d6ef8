// Host-side layout arithmetic of the fused round kernels: the fp32 parameter image and LDS
// layout (MLPDesc) and the bf16 LDS layouts of the train / evaluation kernels (MLPDescB).
// Header-only and free of HIP runtime calls, so the same code the engine uses is compiled into
// a host test binary with AddressSanitizer + UBSan (tests/native/test_layout.cpp) that sweeps
// model shapes and checks every region the kernels index for bounds, overlap and alignment.
#pragma once
#include <algorithm>
#include <cstring>

#include "fl_common.h"

// Activation row stride: roundup16(dim) + 4 floats (16-byte aligned rows, 4 mod 8: with the
// chunk swizzle of fl_kernels.hip (fl_swz) the b128 / b32 MFMA operand patterns are
// bank-conflict free).
inline int fl_pick_ld(int dim) { return ((dim + 15) & ~15) + 4; }

// dims[0..L]: features, hidden sizes, classes.  Fills the dense / image offsets and the fp32
// kernels' LDS layout (floats) for R rows per workgroup.
inline void fl_build_fp32_layout(const int* dims, int L, int R, MLPDesc* d) {
    std::memset(d, 0, sizeof(*d));
    d->L = L;
    int off = 0;
    for (int l = 0; l <= L; ++l) d->dim[l] = dims[l];
    for (int l = 0; l < L; ++l) {
        d->w_off[l] = off;
        off += dims[l] * dims[l + 1];
        d->b_off[l] = off;
        off += dims[l + 1];
    }
    d->P = off;
    // parameter image (fl_common.h): per layer [wrows(N)][ldw(K)] then bias[roundup16(N)]
    int io = 0;
    for (int l = 0; l < L; ++l) {
        d->iw_off[l] = io;
        io += fl_wrows(dims[l + 1]) * fl_ldw(dims[l]);
        d->ib_off[l] = io;
        io += (dims[l + 1] + 15) & ~15;
    }
    d->Pimg = (io + 3) & ~3;
    int lds = 0;
    for (int l = 0; l <= L; ++l) {
        d->ld[l] = fl_pick_ld(dims[l]);
        d->act_off[l] = lds;
        lds += R * d->ld[l];
        lds = (lds + 3) & ~3;
    }
    for (int l = 1; l < L; ++l) {  // backward deltas of the hidden layers
        d->dlt_off[l] = lds;
        lds += R * d->ld[l];
        lds = (lds + 3) & ~3;
    }
    d->cm_off = lds;  // fused evaluation's confusion counters (FL_CM_INTS ints)
    lds += FL_CM_INTS;
    d->img_lds = lds;
    lds += d->Pimg;
    d->lds_floats = lds;
}

// Lagged rounds (FL_EVAL_LAGGED) score the previous round's local model in registers
// (fl_kernels_bf16.hip score_rows_regs) when: one or two hidden layers; the register operands
// fit (features <= 32, with two hidden layers the first <= 64 wide); C <= FL_LAG_MAX_C; the
// logits' K split leaves each upper scoring wave at most FL_LAG_PARTS partials; the training
// forward pass fits the first FL_WAVES - FL_LAG_SPR R/16 waves (hidden tiles are strided over them; the
// logits layer's split K loop and its partial sum must fit them as they are), so the last
// FL_LAG_SPR R/16 waves -- FL_LAG_SPR per 16 rows -- score while the others train; and the LDS holds the
// partials beside the layout.  Otherwise the scoring pass runs before the training pass on the
// whole workgroup.
inline int fl_lag_reg_static_bytes(int R) { return (R / 16) * ((FL_LAG_SPR - 1) * FL_LAG_PARTS * 16 * 16 + 16); }
inline bool fl_lag_reg_ok(const MLPDesc& d, const MLPDescB& e, int R) {
    const int L = d.L, C = d.dim[L];
    const int nw = FL_WAVES - FL_LAG_SPR * (R / 16);
    if ((R != 16 && R != 32) || nw < 1 || (L != 2 && L != 3) || C > FL_LAG_MAX_C) return false;
    if (e.kp[0] > 32 || (L == 3 && e.kp[1] > 64)) return false;
    const int G = e.head_split;
    if (G > nw) return false;
    for (int j = 1; j < FL_LAG_SPR; ++j)
        if (fl_lag_w(G, j + 1) - fl_lag_w(G, j) > FL_LAG_PARTS) return false;
    if (R * C > nw * 64) return false;  // the logits' partial sums (fwd_head_split_bf16) run on thread < R*C
    // the partials ride in static LDS beside the dynamic layout (FL_LDS_DYNAMIC_MAX keeps 2 KB for
    // the kernels' own small statics; ~256 B are taken)
    return e.lds_bytes + fl_lag_reg_static_bytes(R) + 256 <= 160 * 1024;
}

// bf16 LDS layouts (fl_common.h MLPDescB), byte offsets, 16-byte aligned pieces: `e` for the
// train kernel, `ev` for the evaluation kernels (forward pass only), at bank layout `level`.
inline void fl_build_bf16_layout_level(const MLPDesc& d, int R, int level, MLPDescB* e_out, MLPDescB* ev_out) {
    MLPDescB e, ev;
    std::memset(&e, 0, sizeof(e));
    const int L = d.L;
    e.level = level;
    e.wgap = level == 2 ? 128 : 0;
    e.wxor = level == 2 ? 0 : 1;
    for (int l = 0; l <= L; ++l) {
        e.kp[l] = (d.dim[l] + 31) & ~31;
        e.lda[l] = e.kp[l] + (level >= 1 ? 16 : 8);
        if (l < L) e.ldw[l] = e.kp[l] + (level == 2 ? 16 : 8);
    }
    int off = 0;
    auto take = [&](int bytes) { const int o = off; off += (bytes + 15) & ~15; return o; };
    for (int l = 0; l < L; ++l) e.act_off[l] = take(R * e.lda[l] * 2);
    for (int l = 1; l <= L; ++l) e.dlt_off[l] = take(R * e.lda[l] * 2);
    e.logit_off = take(R * FL_LOGIT_LD * 4);
    e.cm_off = take(FL_CM_INTS * 4);
    // split-bf16 forward: lo parts of the layer inputs -- X in its own buffer, the hidden
    // activations in the delta buffers (same [R][lda] shape, free until the backward pass)
    e.alo_off[0] = take(R * e.lda[0] * 2);
    for (int l = 1; l < L; ++l) e.alo_off[l] = e.dlt_off[l];
    // parameter region: W hi images, biases, W lo images (each W size is a multiple of 16
    // bytes, so the lo images sit at one constant offset from their hi images)
    e.param_off = off;
    for (int l = 0; l < L; ++l) e.w_off[l] = take(fl_wrow(e.kp[l + 1], e.ldw[l], e.wgap));
    for (int l = 0; l < L; ++l) e.bias_off[l] = take(e.kp[l + 1] * 4);
    e.wlo_delta = off - e.w_off[0];
    for (int l = 0; l < L; ++l) take(fl_wrow(e.kp[l + 1], e.ldw[l], e.wgap));
    e.param_bytes = off - e.param_off;
    e.lds_bytes = off;
    e.item_base[0] = 0;
    for (int l = 0; l < L; ++l) e.item_base[l + 1] = e.item_base[l] + e.kp[l + 1] * (e.kp[l] >> 3);
    // Evaluation kernels run the forward pass only: their layout has no delta buffers, so the
    // lo parts of the hidden activations get buffers of their own.
    ev = e;
    off = 0;
    for (int l = 0; l < L; ++l) ev.act_off[l] = take(R * e.lda[l] * 2);
    for (int l = 1; l <= L; ++l) ev.dlt_off[l] = -1;
    ev.logit_off = take(R * FL_LOGIT_LD * 4);
    ev.cm_off = take(FL_CM_INTS * 4);
    for (int l = 0; l < L; ++l) ev.alo_off[l] = take(R * e.lda[l] * 2);
    ev.param_off = off;
    for (int l = 0; l < L; ++l) {
        ev.w_off[l] = e.w_off[l] - e.param_off + ev.param_off;
        ev.bias_off[l] = e.bias_off[l] - e.param_off + ev.param_off;
    }
    ev.lds_bytes = ev.param_off + e.param_bytes;
    // Logits layer (one 16-column tile): its K loop is split over up to 16 waves (fixed-order
    // sum of the partial logits) instead of one wave's chain of kp/32 steps, as far as LDS room
    // allows; the same split in both layouts, so training, fused and classic evaluation see
    // bit-identical logits.
    const int C = d.dim[L];
    const int part1 = R * C * 4;
    const int ksteps = e.kp[L - 1] >> 5;
    const int room = (int)FL_LDS_DYNAMIC_MAX - std::max(e.lds_bytes, ev.lds_bytes) - 16;
    int G = std::min(std::min(ksteps, 16), std::max(1, room / part1));
    if (G < 2) G = 1;
    e.head_split = ev.head_split = G;
    if (G > 1) {
        e.part_off = e.lds_bytes;
        e.lds_bytes += (G * part1 + 15) & ~15;
        ev.part_off = ev.lds_bytes;
        ev.lds_bytes += (G * part1 + 15) & ~15;
    }
    e.lag_reg = ev.lag_reg = fl_lag_reg_ok(d, e, R) ? 1 : 0;
    *e_out = e;
    *ev_out = ev;
}

// The most conflict-free level whose train and evaluation layouts fit the CU's LDS (level 0
// when none fits: the engine then refuses this R).
inline void fl_build_bf16_layout(const MLPDesc& d, int R, MLPDescB* e_out, MLPDescB* ev_out) {
    for (int level = 2; level >= 0; --level) {
        fl_build_bf16_layout_level(d, R, level, e_out, ev_out);
        if (std::max(e_out->lds_bytes, ev_out->lds_bytes) <= (int)FL_LDS_DYNAMIC_MAX) return;
    }
}
