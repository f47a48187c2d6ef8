// Shared host/device declarations of the fused federated-round engine.
//
// One client per GPU keeps everything resident: the local shard, the parameters, the Adam
// moments (which persist across rounds), a per-block gradient slab, and a small
// device-side round state that carries the early-stopping rule
// (FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:181-192) so the host never has to
// read metrics back to decide whether to continue.
//
// Parameter "image" layout.  Every parameter-shaped device buffer (global/comm, local, m, v)
// stores, per layer l, W_l ([N][K], torch Linear layout) as fl_wrows(N) rows of fl_ldw(K)
// floats followed by b_l padded to roundup16(N), all padding zero; W_l[n][k] sits at column
// k ^ fl_swz(n) of row n (the fp32 kernels' LDS chunk swizzle, fl_kernels.hip).  The image is
// exactly the LDS image the fp32 kernels compute from, so staging a model into LDS is one
// contiguous float4 copy, and every MFMA operand read of a 16x16 tile / 16-deep k chunk is in
// bounds and reads zeros in the padding (no predication, no exec-mask branches in inner loops).  The dense
// reference layout (named_parameters() order: model.0.weight, model.0.bias, ...; C:93-99)
// exists only at the API boundary (get/set weights, checkpoints) and in the gradient slab.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FL_MAX_LAYERS 4
#define FL_MAX_CLASSES 16
#define FL_MAX_WORLD 64
// Dynamic LDS a fused-kernel workgroup may request: the CU's 160 KiB minus room for the
// kernels' small static __shared__ objects (round state, counters).
#define FL_LDS_DYNAMIC_MAX (160 * 1024 - 2048)
// Threads of a fused-kernel workgroup (overridable for variant builds: -DFL_THREADS=...).
#ifndef FL_THREADS
#define FL_THREADS 1024
#endif
#define FL_WAVES (FL_THREADS / 64)
// Lagged rounds scored in registers (fl_layout.h fl_lag_reg_ok): FL_LAG_SPR waves per 16-row
// group split the last hidden layer; each upper one hands at most FL_LAG_PARTS logits partials
// (C <= 4 classes) to the group's first wave through LDS.
#ifndef FL_LAG_SPR
#define FL_LAG_SPR 3
#endif
#define FL_LAG_PARTS (FL_LAG_SPR == 2 ? 4 : 2)
#define FL_LAG_MAX_C 4
// logits part range of scoring wave j of a group (parts [fl_lag_w(G, j), fl_lag_w(G, j + 1)))
__host__ __device__ inline int fl_lag_w(int G, int j) { return G - ((FL_LAG_SPR - j) * G) / FL_LAG_SPR; }

// ldw = roundup16(K) + 4 (4 mod 8 floats): 16-byte aligned rows; with the chunk swizzle
// (fl_swz below) the rows of every gfx950 ds_read_b128 lane group land on distinct 16-byte
// bank slots.
__host__ __device__ inline int fl_ldw(int K) { return ((K + 15) & ~15) + 4; }
__host__ __device__ inline int fl_wrows(int N) { return (N + 15) & ~15; }
// fp32 LDS / image chunk swizzle: row r keeps logical column k < roundup16(width) at column
// k ^ fl_swz(r) -- the 4-float chunks of rows 4..11 (mod 16) trade places in pairs
// (fl_kernels.hip; models/mlp.py mirrors it).
__host__ __device__ inline int fl_swz(int r) { return ((r + 4) & 8) >> 1; }

struct MLPDesc {
    int L;                            // number of Linear layers
    int dim[FL_MAX_LAYERS + 1];       // dim[0] = features, dim[L] = classes
    int ld[FL_MAX_LAYERS + 1];        // LDS leading dimension (floats) per activation buffer
    int act_off[FL_MAX_LAYERS + 1];   // LDS float offset of each activation buffer (R rows)
    int dlt_off[FL_MAX_LAYERS + 1];   // LDS float offset of the backward delta of hidden layer l
    int w_off[FL_MAX_LAYERS];         // dense (reference) offset of W_l
    int b_off[FL_MAX_LAYERS];         // dense offset of b_l
    int P;                            // dense parameter count
    int iw_off[FL_MAX_LAYERS];        // image offset of W_l
    int ib_off[FL_MAX_LAYERS];        // image offset of b_l
    int Pimg;                         // image floats (multiple of 4)
    int img_lds;                      // LDS float offset of the staged image
    int cm_off;                       // LDS float offset of the C x C int confusion counters
    int lds_floats;                   // LDS floats needed per block
};

// bf16 LDS layout of the fused kernels (fl_kernels_bf16.hip).  All offsets are BYTES into
// the dynamic LDS window.  Every fan-in dimension is padded to kp = roundup32(dim) (one
// v_mfma_f32_16x16x32_bf16 k-step per 32).  W_l has kp[l+1] rows (the dgrad contraction
// runs over its padded fan-out), activations / deltas have R rows.  Transposed operands (wgrad
// over rows, dgrad over W's rows) are read with ds_read_b64_tr_b16 from the same images.
//
// Bank conflicts (64 banks x 4 B; ds_read_b128 serves 16 lanes per LDS cycle,
// ds_read_b64_tr_b16 32 lanes; tests/native/test_layout.cpp models both).  Three layout
// levels, the best that fits the CU's LDS (fl_layout.h):
//   * activation / delta rows lda = kp + 16 elements (levels 1, 2): a row stride of an odd
//     multiple of 32 bytes, on which a b128 group (16 rows x 16 B) and a transposed read of 8
//     CONSECUTIVE rows x 32 B both tile the 256-byte bank period exactly.  wgrad takes its 32
//     row-k's as runs 4g..4g+3 / 16+4g..16+4g+3 per 16-lane group g (same order in both
//     operands), so each transposed read covers 8 consecutive rows.  Level 0: kp + 8.
//   * W images: row n at fl_wrow(n) = n*ldw*2 + (n/8)*wgap bytes, its 16-byte chunk c stored
//     at chunk c ^ (wxor * bit 3 of n); lane lr of a forward tile reads W row
//     fl_fwd_col(lr) = (lr + 4) & 15 and produces that output column.  Level 2: ldw = kp + 16,
//     wgap 128, wxor 0 -- dgrad's transposed reads of rows {0-3, 8-11} (k-runs tied to the b128
//     rows of the delta operand) land half a bank period apart, every read is conflict free.
//     Levels 0/1: ldw = kp + 8, no gap, wxor 1 -- the forward reads are conflict free, dgrad's
//     transposed W reads 2-way (the 10 KB of gaps and pads do not fit beside R = 32 rows of a
//     (50, 200) model).
//
// Split-bf16 forward ("bf16x3").  Every forward pass computes z = a.W^T as
// a_hi.W_hi^T + (a_lo.W_hi^T + a_hi.W_lo^T) with x_hi = bf16(x), x_lo = bf16(x - x_hi), fp32
// accumulation: ~16 significant bits per product instead of 8.  The backward pass stays plain
// bf16 (hi parts).  Reason: the reference's early-stop rule (C:181-192, atol 1e-4 on 8000-row
// accuracies) needs 10 rounds without a single prediction flip; with 8-bit scoring every
// bf16 rounding step of a changing weight flips borderline rows and the rule never fires
// (tools/bf16_es_emulate.py: split-bf16 forward stops at rounds 175-238, the fp32 oracle at
// 157-227, the reference at 149-243).  The lo images of the weights sit in the parameter
// region `wlo_delta` bytes after their hi images (same layout); the lo parts of the layer
// inputs live in `alo_off` buffers (X lo: its own buffer; hidden layers: the backward delta
// buffers, unused during the forward pass).
struct MLPDescB {
    int kp[FL_MAX_LAYERS + 1];        // roundup32(dim[l])
    int lda[FL_MAX_LAYERS + 1];       // row stride (elements) of act_l, D_l: kp[l] + 16 (level 0: + 8)
    int ldw[FL_MAX_LAYERS];           // row stride (elements) of W_l: kp[l] + 16 (level 2) or + 8
    int wgap;                         // bytes after every 8 W rows (level 2: 128)
    int wxor;                         // W chunk swizzle (levels 0/1: 1)
    int level;                        // bank layout level (2 = conflict free, see above)
    int w_off[FL_MAX_LAYERS];         // W_l  bf16 kp[l+1] rows, fl_wbyte() positions (hi parts)
    int bias_off[FL_MAX_LAYERS];      // b_l  fp32 [kp[l+1]] (zero padded)
    int wlo_delta;                    // W_l lo parts at w_off[l] + wlo_delta (same layout)
    int act_off[FL_MAX_LAYERS + 1];   // act_l bf16 [R][lda[l]]   (l < L), hi parts
    int alo_off[FL_MAX_LAYERS + 1];   // act_l lo parts bf16 [R][lda[l]] (l < L; forward pass only)
    int dlt_off[FL_MAX_LAYERS + 1];   // D_l  bf16 [R][lda[l]]    (1 <= l <= L): dLoss/dz_l
    int logit_off;                    // fp32 [R][FL_LOGIT_LD] classifier logits (16 columns)
    int head_split;                   // logits layer: K split over this many waves (1 = one wave)
    int part_off;                     // ... their fp32 partial logits [head_split][R][C]
    int cm_off;                       // int [16][16] confusion counters (fused evaluation)
    int item_base[FL_MAX_LAYERS + 1]; // packing: prefix sums of the 8-element items of each W_l
    int param_off;                    // start of the parameter region (all W_l hi, all b_l, all W_l lo):
    int param_bytes;                  // it is stored pre-packed in global memory and staged by a copy
    int lds_bytes;
    int lag_reg;                      // 1: lagged rounds score in registers (fl_layout.h fl_lag_reg_ok)
};

// Packed bf16 W images (see the bank notes above): byte offset of row n (fl_wrow(kp rows) =
// image bytes), the chunk swizzle of row n, the byte position of element (n, k), and the W
// row / output column that lane lr of a forward tile computes.
__host__ __device__ inline int fl_wrow(int n, int ldw, int wgap) { return n * ldw * 2 + (n >> 3) * wgap; }
__host__ __device__ inline int fl_wswz(int n, int wxor) { return ((n >> 3) & 1) * wxor; }
__host__ __device__ inline int fl_wbyte(const MLPDescB& e, int l, int n, int k) {
    return fl_wrow(n, e.ldw[l], e.wgap) + ((((k >> 3) ^ fl_wswz(n, e.wxor)) << 4) | ((k & 7) << 1));
}
__host__ __device__ inline int fl_fwd_col(int lr) { return (lr + 4) & 15; }
// The 4 accumulator rows of an MFMA lane (4g + j, 16-lane group g) go to LDS in 4 writes; in
// write t a lane of an odd group writes row 4g + ((t + 1) & 3), so the two 16-lane groups of a
// 32-lane write half are 5 or 1 rows apart instead of 4 (4 rows = 0 mod the 128-byte write
// bank period at these strides).
__host__ __device__ inline int fl_out_row(int lg, int t) { return 4 * lg + ((t + (lg & 1)) & 3); }
// Logit rows: 17 floats apart (one row per lane in the loss epilogue: distinct banks).
#define FL_LOGIT_LD 17

struct FLConfig {
    int R;              // rows per workgroup (16 or 32)
    int n_rows;         // local training rows
    float inv_n;        // 1 / n_rows  (CrossEntropyLoss 'mean', C:43)
    int world;
    int rank;
    float agg_scale;    // n_rank / N_total (sample-size-weighted FedAvg, C:110-116)
    int slab_stride;    // floats per slab row (dense P + loss slot, padded)
    int n_slabs;        // workgroups of the train kernel = ceil(n_rows / R)
    int slab_f16;       // bf16 kernels: the slab holds fp16 partial SUMS (the 1/n is applied by
                        // Adam after the fp32 reduction; fl_device.h slab_store_h)
    int tail_off;       // == Pimg: start of the per-rank metric tail in the comm buffer
    int tail_stride;    // C*C confusion counts + 1 loss slot
    int tail_len;       // world * tail_stride
    int lag_off;        // > 0: start of the lag region A (tail_len floats, FL_EVAL_LAGGED)
    int plain_fwd;      // bf16, several clients, register scoring: the TRAINING forward pass is plain
                        // bf16 (a_hi.W_hi) and stages only the hi images -- every scoring pass is a
                        // separate split-bf16 forward there (fl_kernels_bf16.hip)
    int split_score;    // lagged rounds score on n_slabs workgroups of their own (train kernel LAG 3)
                        // instead of on waves of the training workgroups (LAG 2): small shards
    int local_steps;    // optimizer steps per round (reference: 1 full-batch step, C:63-73)
    // optimizer (torch.optim.Adam + StepLR, C:44-46); scalars kept in double like torch
    double lr0;
    double gamma;
    int step_size;
    double beta1;
    double beta2;
    float omb1;         // (float)(1 - beta1)  lerp weight
    float omb2;         // (float)(1 - beta2)  addcmul value
    float beta2f;       // (float)beta2
    float eps;
    float weight_decay; // L2 on the gradient (torch Adam weight_decay / sklearn alpha)
    float prox_mu;      // FedProx proximal coefficient (0 = FedAvg)
    // early stopping (C:122, C:181-192)
    int es_enabled;
    int patience;
    double atol;
    double rtol;
    int max_rounds;
    int metric_mode;    // 0 = mean of per-client metrics (C:169), 1 = pooled confusion (S:130)
};

// Device-resident round state; double-buffered by round parity so every workgroup of the
// train kernel can recompute the stop decision from an immutable input copy.
struct FLState {
    int next_round;     // index of the next round to run
    int finalized;      // rounds whose metrics have been folded into the history
    int stopped;        // early-stop signal (C:132-136 / C:189)
    int live;           // this launch's round is live (not past the stop)
    int cur_round;      // index of the round running now (valid when live)
    int count;          // patience counter (termination_count, C:125)
    int has_prev;
    int stop_round;     // round index at which the stop took effect (-1 = none)
    unsigned calls;     // Adam-fused FedAvg exchanges done (call index of the chunk flags, peer_device.h)
    // 1: this round's fold found a stop triggered by round next_round - 2 (lag region A folded one
    // round late: lagged rounds over an external all-reduce with early stopping), so round
    // next_round - 1 ran past the stop.  Its output is discarded: the round republishes the image
    // still held by its own comm buffer -- round next_round - 2's all-reduced output (the comm
    // buffer of round q is the output buffer of round q - 2) -- instead of its input.
    int late;
    double prev[4];     // prev_metric (C:126)
};

struct FLBuffers {
    const float* X;     // [n_rows, dim0] row-major, device resident
    const int* y;       // [n_rows]
    float* slab;        // [n_slabs, slab_stride] dense gradient partials (fp32; slab_f16: fp16 in the
                        // first P halves of each row, the loss partial stays the fp32 at [P])
    float* local;       // [Pimg] post-step local weights (evaluated, C:148)
    float* m;           // [Pimg] Adam exp_avg
    float* v;           // [Pimg] Adam exp_avg_sq
    double* hist_global;  // [max_rounds, 4]
    double* hist_rank;    // [max_rounds, world, 4]
    float* hist_loss;     // [max_rounds] mean CE over clients
    unsigned long long* dbg;  // optional [blocks, 16] s_memrealtime phase stamps (profiling)
    char* pk_global;    // bf16 mode: packed LDS-layout image of the round's input weights
    char* pk_local;     // bf16 mode: packed LDS-layout image of the local (post-Adam) weights
    // Adam + StepLR scalars per optimizer step slot t = 1 .. max_rounds * local_steps (slot of
    // round r, local step ls: r * local_steps + ls + 1), computed on the host in double exactly
    // as torch does (python float pow): [t-1] = {step_size, sqrt(bias_correction2)} rounded to
    // fp32, with the bias corrections of the CLIENT'S OWN Adam step count (= t without client
    // sampling) and the LR of the round.  A table lookup instead of three double pow() on the
    // Adam kernel's critical path.
    const float* sched;
    // Per-round FedAvg table [max_rounds][4] = {this client's aggregation weight (n_i / sum of
    // the round's sampled n_j; 0 when not sampled), sampled-client count, sampled-rank bitmask
    // bits 0-31, bits 32-63 (bit patterns stored in the float slots)}.  Full participation:
    // {n_i / N, world, all ones}.  Built on the host from the seeded per-round client sample
    // (fedmi/fl/engine.py participants()), identical on every rank.
    const float* rtab;
    float* cnt;         // FL_EVAL_LAGGED: confusion counts of the previous round's local model
    float* lbuf;        // FL_EVAL_LAGGED: the previous round's loss, published one round later
    // Late fold (FLState::late; lagged rounds over an external all-reduce with early stopping):
    // [local | m | v] (3 x Pimg floats) and the packed local image (undo_pk_bytes) as they were
    // before the last live round's first optimizer step, written by adam_update; a round found
    // to have run past the stop restores them, so the local model and the Adam moments match a
    // run that stopped in time.  nullptr: no round can be discarded.
    float* undo;
    int undo_pk_bytes;
    int* sat;           // optional: set to 1 by the Adam kernel when an fp16 slab partial it reads is
                        // saturated (|x| = 65504, slab_store_h's clamp) or not finite
};

// Evaluation placement of a round (`mode` of the train kernels).
//   FL_EVAL_CLASSIC : the train kernel folds the previous round's metrics into the state at
//                     its start; a separate eval kernel scores the post-step model.
//   FL_EVAL_FUSED   : one client (FedAvg is the identity, so the round's input weights ARE
//                     the previous round's post-step local model): the train kernel's own
//                     forward pass yields the previous round's confusion counts (argmax in
//                     the loss epilogue) and the Adam kernel folds them and decides whether
//                     this round is live.  No eval kernel.
//   FL_EVAL_FUSED_SKIP : as FUSED, but the previous round's counts are already in the tail
//                     (that round ran classic); the train kernel only trains.
#define FL_EVAL_CLASSIC 0
#define FL_EVAL_FUSED 1
#define FL_EVAL_FUSED_SKIP 2
//   FL_EVAL_LAGGED  : several clients: the train kernel of round r first scores round r-1's
//                     post-step LOCAL model (a forward pass on the staged local image, before
//                     the round's own weights replace it in LDS) into the local count buffer;
//                     the Adam kernel publishes those counts (+ round r-1's loss) in region A
//                     of round r's exchange, so no round needs a separate evaluation kernel.
//                     With the Adam-fused exchange region A is exchanged and folded inside
//                     round r's Adam kernel (in time for early stopping); riding an external
//                     all-reduce (RCCL) it is folded one round later, by round r+1's Adam
//                     kernel -- with early stopping round r runs before round r-1's stop is
//                     known and is then discarded bit-exactly (FLState::late).
#define FL_EVAL_LAGGED 3
// Metric regions of an all-reduced comm buffer that a fold consumes (fl_device.h).
#define FL_FOLD_A 1  // lag region: round next_round - 2
#define FL_FOLD_B 2  // tail region: round next_round - 1
// LDS confusion-counter region of the train kernels: C*C counters + a "score rows" flag,
// padded to a multiple of 16 bytes.
#define FL_CM_FLAG (FL_MAX_CLASSES * FL_MAX_CLASSES)
#define FL_CM_INTS (FL_CM_FLAG + 4)

// Trial batches (BASELINE config 5, fedmi/hpo/fed_sweep.py): K engines of the same shape --
// same layer sizes, R, rows (one client's shard), dtype -- that differ in hyperparameters (lr,
// local steps, FedProx mu, ...) advance in lock-step, and every kernel of a round runs ONCE for
// all of them with a trial grid dimension (blockIdx.y = trial) instead of K launches.  Each
// trial's configuration, buffers and the pointer bases its launches refer to sit in a device
// table; a launch names each pointer argument as (base slot, byte offset), the same for every
// trial of the batch (the recording engine checks that, fl_engine.cpp TrialBatch).
#define FL_TB_BASES 8
enum { FL_TB_PBUF0 = 0, FL_TB_PBUF1, FL_TB_ST0, FL_TB_ST1, FL_TB_LOCAL, FL_TB_LAG, FL_TB_PKG, FL_TB_PKL };
struct FLTrialDesc {
    FLConfig c;
    FLBuffers b;
    char* base[FL_TB_BASES];
};
struct FLSel {
    int base;        // FL_TB_* slot, -1 = nullptr
    int pad;
    long long off;   // bytes
};
__host__ __device__ inline char* fl_sel(const FLTrialDesc& t, FLSel s) {
    return s.base < 0 ? nullptr : t.base[s.base] + s.off;
}

struct PeerArgs;  // peer_device.h
struct PeerPack;
// Launchers (fl_kernels.hip). `pg` = image the round trains from (the previous round's
// all-reduced comm buffer), `comm` = buffer this round publishes into (Pimg + tail floats).
// `cm_out` = this rank's confusion slots of pg's tail (FL_EVAL_FUSED only).
hipError_t fl_launch_train(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                           const float* pg, const FLState* st_in, FLState* st_out,
                           int local_step, hipStream_t s, int mode = FL_EVAL_CLASSIC,
                           float* cm_out = nullptr, int fold_mask = FL_FOLD_B);
// `st` = state the step runs under; with `fold` (FL_EVAL_FUSED rounds, first local step) it
// is the previous round's state: every block folds pg's tail into it, block 0 writes the
// round's state to `st_out`.
hipError_t fl_launch_adam(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                          const float* pin, const float* anchor, float* comm,
                          const FLState* st, int local_step, hipStream_t s,
                          const MLPDescB* e = nullptr, FLState* st_out = nullptr, int fold = 0,
                          int tail_a = 0, int fold_mask = FL_FOLD_B, const PeerArgs* peer = nullptr, int wx = 0,
                          int afold = 0);
// (fl_adam_local.hip: the Adam kernel without the in-kernel exchange; fl_launch_adam picks it)
hipError_t fl_launch_adam_local(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                                const float* anchor, float* comm, const FLState* st, int local_step,
                                const MLPDescB& e, int pack, FLState* st_out, int fold, int tail_a, int fold_mask,
                                hipStream_t s);
// (fl_adam_local.hip: the Adam kernel for exchanges on LL chunks)
hipError_t fl_launch_adam_ll(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                             const float* anchor, float* comm, const FLState* st, int local_step, const MLPDescB& e,
                             int pack, FLState* st_out, int fold, int tail_a, int fold_mask, const PeerArgs& pa,
                             int xchg, int afold, hipStream_t s);
hipError_t fl_launch_eval(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                          const float* params, float* comm, const FLState* st, hipStream_t s);
// `prev_out` (may be null): the other parameter buffer -- the round before pg's output.  When
// the fold finds a late stop (FLState::late) pg's image is replaced by it.
hipError_t fl_launch_finalize(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                              float* pg, const FLState* st_in, FLState* st_out,
                              hipStream_t s, int mask = FL_FOLD_B, const float* prev_out = nullptr);
// bf16-operand variants (split-bf16 forward, bf16 backward, fp32 accumulate, fp32 master
// weights / slab / Adam state).
hipError_t fl_launch_train_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                                const float* pg, const FLState* st_in, FLState* st_out, int local_step,
                                hipStream_t s, bool stage_local = false, int mode = FL_EVAL_CLASSIC,
                                float* cm_out = nullptr, int fold_mask = FL_FOLD_B);
hipError_t fl_launch_eval_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                               const float* params, float* comm, const FLState* st, hipStream_t s);
hipError_t fl_set_lds_limit_bf16(size_t bytes);
// fp32 parameter image -> packed bf16 LDS-layout parameter region (MLPDescB)
// Local evaluation + FedAvg in one kernel (world > 1 with the one-shot xGMI all-reduce,
// peer_device.h): the all-reduce of the call described by `a` runs in extra blocks beside
// the evaluation of `params` into this rank's tail slot of `comm` (the call's send buffer).
hipError_t fl_launch_eval_fedavg(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* params,
                                 float* comm, const FLState* st, const PeerArgs& a, const PeerPack& pk,
                                 hipStream_t s);
hipError_t fl_launch_eval_fedavg_bf16(const MLPDesc& d, const MLPDescB& e, const FLConfig& c, const FLBuffers& b,
                                      const float* params, float* comm, const FLState* st, const PeerArgs& a,
                                      const PeerPack& pk, hipStream_t s);
hipError_t fl_launch_pack_bf16(const MLPDesc& d, const MLPDescB& e, const float* params, char* out, hipStream_t s);
// Batched launches of K trials (FLTrialDesc table `T`, K = gridDim.y): the same kernels, every
// pointer argument a selector into the trial's bases.  `cm` of the train launch and `comm` of
// the eval launch follow the single-trial launchers (the eval's confusion slots are derived
// from `comm` per trial).
hipError_t fl_launch_train_batch(const MLPDesc& d, int R, int n_slabs, const FLTrialDesc* T, int K, FLSel pg,
                                 FLSel si, FLSel so, int ls, int mode, FLSel cm, int fold_mask, hipStream_t s);
hipError_t fl_launch_train_bf16_batch(const MLPDesc& d, const MLPDescB& e, int R, int n_slabs, const FLTrialDesc* T,
                                      int K, FLSel pg, FLSel si, FLSel so, int ls, int stage_local, int mode, FLSel cm,
                                      int fold_mask, hipStream_t s, int plain = 0);
hipError_t fl_launch_adam_batch(const MLPDesc& d, const MLPDescB* e, const FLTrialDesc* T, int K, FLSel pin,
                                FLSel anchor, FLSel comm, FLSel st, int local_step, FLSel st_out, int fold, int tail_a,
                                int fold_mask, hipStream_t s);
hipError_t fl_launch_eval_batch(const MLPDesc& d, int R, int n_rows, const FLTrialDesc* T, int K, FLSel params,
                                FLSel comm, FLSel st, hipStream_t s);
hipError_t fl_launch_eval_bf16_batch(const MLPDesc& d, const MLPDescB& e, int R, int n_rows, const FLTrialDesc* T,
                                     int K, FLSel params, FLSel comm, FLSel st, hipStream_t s);
hipError_t fl_launch_pack_bf16_batch(const MLPDesc& d, const MLPDescB& e, const FLTrialDesc* T, int K, FLSel params,
                                     FLSel out, hipStream_t s);
hipError_t fl_launch_finalize_batch(const MLPDesc& d, const FLTrialDesc* T, int K, FLSel pg, FLSel si, FLSel so,
                                    int mask, hipStream_t s);
// Stand-alone forward + confusion on an arbitrary row set (held-out evaluation).
hipError_t fl_launch_confusion(const MLPDesc& d, int R, const float* X, const int* y, int n_rows,
                               const float* params, float* cm_out, hipStream_t s);
// Fill a device shard with synthetic income-shaped rows (Philox4x32-10).
hipError_t fl_launch_synth(float* X, int* y, long long n_rows, int n_features,
                           unsigned long long seed, unsigned long long row_offset,
                           const float* teacher_w1, const float* teacher_w2, int teacher_hidden,
                           hipStream_t s, float label_noise = 0.f);
// Hold stream `s` for `us` microseconds (one sleeping wave; FLEngine::trace).
hipError_t fl_launch_gate(double us, hipStream_t s);
