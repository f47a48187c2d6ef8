// Host test of the fused kernels' index arithmetic (fedmi/ops/csrc/fl_layout.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host (tests/test_native_layout.py).
//
// For every model shape the engine accepts, it replays -- on the host, lane by lane -- the LDS
// addresses the bf16 / fp32 train and evaluation kernels compute (fl_kernels_bf16.hip,
// fl_kernels.hip: staging, split-bf16 forward, split-K logits, weight / input gradients, the
// Adam kernel's packed-image stores, the peer epilogue's pack) and checks that each access stays
// inside the region it is meant for, that regions do not overlap, and that the layouts fit the
// CU's LDS.  Every region is backed by its own heap allocation of exactly its size, and each
// simulated access touches those bytes, so an out-of-region index is also caught by ASan.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "fl_layout.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                      \
    do {                                                      \
        if (!(cond)) {                                        \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                \
            std::fprintf(stderr, "\n");                       \
            if (++g_fail > 20) std::exit(1);                  \
        }                                                     \
    } while (0)

// One LDS region [off, off + bytes) backed by an exact-size allocation.
struct Region {
    std::string name;
    int off, bytes;
    std::vector<unsigned char> mem;
};

struct Lds {
    int total;
    std::vector<Region> regs;
    void add(const std::string& n, int off, int bytes) {
        CHECK(off >= 0 && bytes >= 0 && off + bytes <= total, "%s [%d, %d) outside LDS %d", n.c_str(), off, off + bytes,
              total);
        CHECK(off % 16 == 0, "%s offset %d not 16-byte aligned", n.c_str(), off);
        regs.push_back({n, off, bytes, std::vector<unsigned char>((size_t)bytes)});
    }
    // touch bytes [a, a + n) of region `name` (relative to LDS 0)
    void touch(const std::string& name, long a, int n) {
        for (auto& r : regs)
            if (r.name == name) {
                CHECK(a >= r.off && a + n <= r.off + r.bytes, "access [%ld, %ld) outside %s [%d, %d)", a, a + n,
                      name.c_str(), r.off, r.off + r.bytes);
                if (a >= r.off && a + n <= r.off + r.bytes)
                    for (int i = 0; i < n; ++i) r.mem[(size_t)(a - r.off + i)] ^= 1;
                return;
            }
        CHECK(false, "no region %s", name.c_str());
    }
    void no_overlap(const std::vector<std::string>& names) {
        for (size_t i = 0; i < names.size(); ++i)
            for (size_t j = i + 1; j < names.size(); ++j) {
                const Region *a = nullptr, *b = nullptr;
                for (auto& r : regs) {
                    if (r.name == names[i]) a = &r;
                    if (r.name == names[j]) b = &r;
                }
                if (!a || !b) continue;
                CHECK(a->off + a->bytes <= b->off || b->off + b->bytes <= a->off, "%s overlaps %s", a->name.c_str(),
                      b->name.c_str());
            }
    }
};

static std::string nm(const char* s, int l) { return std::string(s) + std::to_string(l); }

// gfx950 LDS bank model (64 banks x 4 B; MI355X_MICROARCH.md, LDS): extra LDS cycles of one
// wave-wide read.  ds_read_b128 is served in 4 lane groups of 16, ds_read_b64 /
// ds_read_b64_tr_b16 in 2 groups of 32; within a group each additional distinct dword on a
// bank costs one cycle.
static int extra_cycles(const long* addr, int bytes) {
    static const int g128[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    const int ngroups = bytes == 16 ? 4 : 2, glen = 64 / ngroups;
    int cycles = 0;
    for (int g = 0; g < ngroups; ++g) {
        std::map<int, std::vector<long>> bank;
        for (int i = 0; i < glen; ++i) {
            const int lane = bytes == 16 ? g128[g][i] : g * 32 + i;
            for (int w = 0; w < bytes / 4; ++w) {
                const long dw = addr[lane] / 4 + w;
                auto& v = bank[(int)(dw % 64)];
                bool seen = false;
                for (long x : v) seen = seen || x == dw;
                if (!seen) v.push_back(dw);
            }
        }
        int worst = 0;
        for (auto& kv : bank) worst = std::max(worst, (int)kv.second.size());
        cycles += worst;
    }
    return cycles - ngroups;
}

// Bank conflicts of the MFMA operand reads of the bf16 train kernel (split-bf16 forward: act /
// act-lo / W / W-lo b128; wgrad: transposed reads of D and act; dgrad: transposed reads of W,
// b128 reads of D), replayed per wave instruction.  Returns the extra cycles (expected 0).
// 2-byte / 4-byte accesses (ds_write_b16, ds_read_u16, ds_read_b32): 2 groups of 32 lanes,
// bank (a/4) mod 32; only the first `active` lanes take part.
static int extra_cycles32(const long* addr, int active) {
    int cycles = 0, groups = 0;
    for (int g = 0; g < 2; ++g) {
        std::map<int, std::vector<long>> bank;
        for (int lane = g * 32; lane < std::min(active, g * 32 + 32); ++lane) {
            const long dw = addr[lane] / 4;
            auto& v = bank[(int)(dw % 32)];
            bool seen = false;
            for (long x : v) seen = seen || x == dw;
            if (!seen) v.push_back(dw);
        }
        if (bank.empty()) continue;
        int worst = 0;
        for (auto& kv : bank) worst = std::max(worst, (int)kv.second.size());
        cycles += worst;
        ++groups;
    }
    return cycles - groups;
}

struct BankStats {
    long act = 0, wfwd = 0, wdgrad = 0;  // extra cycles: activation / delta reads, W forward, W dgrad
    long st = 0;                         // activation / delta stores, ReLU-mask and logit reads
};
static BankStats bank_conflicts_bf16(const MLPDesc& d, const MLPDescB& e, int R) {
    const int L = d.L, RT = R / 16;
    BankStats st;
    long* extra = &st.act;
    long a[64];
    auto run = [&](int bytes, auto&& f) {
        for (int lane = 0; lane < 64; ++lane) a[lane] = f(lane & 15, lane >> 4);
        *extra += extra_cycles(a, bytes);
    };
    for (int l = 0; l < L; ++l) {
        const int lda = e.lda[l], ksteps = e.kp[l] >> 5;
        const bool last = l + 1 == L;
        const int ntiles = last ? 1 : e.kp[l + 1] >> 4;
        for (int nt = 0; nt < ntiles; ++nt)
            for (int ks = 0; ks < ksteps; ++ks) {
                extra = &st.wfwd;
                for (int lo = 0; lo < 2; ++lo)
                    run(16, [&](int lr, int lg) {
                        return (long)e.w_off[l] + lo * e.wlo_delta + fl_wbyte(e, l, nt * 16 + fl_fwd_col(lr), 32 * ks + 8 * lg);
                    });
                extra = &st.act;
                for (int rt = 0; rt < RT; ++rt)
                    run(16, [&](int lr, int lg) { return (long)e.act_off[l] + (lr * lda + 8 * lg) * 2 + rt * 16 * lda * 2 + 64 * ks; });
            }
    }
    for (int l = L - 1; l >= 0; --l) {
        const int ldd = e.lda[l + 1], lda = e.lda[l];
        const int otiles = (d.dim[l + 1] + 15) >> 4, itiles = (d.dim[l] + 15) >> 4;
        for (int ot = 0; ot < otiles; ++ot)
            for (int it = 0; it < itiles; ++it)
                for (int h = 0; h < (RT >= 2 ? RT / 2 : 1); ++h)
                    for (int q = 0; q < (RT >= 2 ? 2 : 1); ++q) {
                        auto row = [&](int lr, int lg) { return RT >= 2 ? 32 * h + 4 * lg + (lr >> 2) + 16 * q : 4 * lg + (lr >> 2); };
                        run(8, [&](int lr, int lg) { return (long)e.dlt_off[l + 1] + (row(lr, lg) * ldd + ot * 16 + 4 * (lr & 3)) * 2; });
                        run(8, [&](int lr, int lg) { return (long)e.act_off[l] + (row(lr, lg) * lda + it * 16 + 4 * (lr & 3)) * 2; });
                    }
        if (l == 0) continue;
        for (int it = 0; it < (e.kp[l] >> 4); ++it)
            for (int os = 0; os < (e.kp[l + 1] >> 5); ++os) {
                extra = &st.wdgrad;
                for (int q = 0; q < 2; ++q)
                    run(8, [&](int lr, int lg) {
                        return (long)e.w_off[l] + fl_wbyte(e, l, 32 * os + 8 * lg + (lr >> 2) + 4 * q, it * 16 + 4 * (lr & 3));
                    });
                extra = &st.act;
                for (int rt = 0; rt < RT; ++rt)
                    run(16, [&](int lr, int lg) { return (long)e.dlt_off[l + 1] + (lr * ldd + 8 * lg) * 2 + rt * 16 * ldd * 2 + os * 64; });
            }
    }
    // 2-byte stores of the forward outputs / input gradients (+ the mask reads at the same
    // addresses), rows written in the fl_out_row order; the loss epilogue's logit reads
    auto run32 = [&](int active, auto&& f) {
        for (int lane = 0; lane < 64; ++lane) a[lane] = f(lane);
        st.st += extra_cycles32(a, active);
    };
    for (int l = 0; l + 1 < L; ++l)
        for (int nt = 0; nt < (e.kp[l + 1] >> 4); ++nt)
            for (int rt = 0; rt < RT; ++rt)
                for (int t = 0; t < 4; ++t)
                    run32(64, [&](int lane) {
                        return (long)e.act_off[l + 1] +
                               ((rt * 16 + fl_out_row(lane >> 4, t)) * e.lda[l + 1] + nt * 16 + fl_fwd_col(lane & 15)) * 2;
                    });
    for (int l = L - 1; l >= 1; --l)
        for (int it = 0; it < (e.kp[l] >> 4); ++it)
            for (int rt = 0; rt < RT; ++rt)
                for (int t = 0; t < 4; ++t)
                    run32(64, [&](int lane) {
                        return (long)e.dlt_off[l] + ((rt * 16 + fl_out_row(lane >> 4, t)) * e.lda[l] + it * 16 + (lane & 15)) * 2;
                    });
    for (int k = 0; k < d.dim[L]; ++k) run32(R, [&](int lane) { return (long)e.logit_off + (lane * FL_LOGIT_LD + k) * 4; });
    return st;
}

// The bf16 kernels' accesses (train layout when `train`, evaluation layout otherwise).
static void check_bf16(const MLPDesc& d, const MLPDescB& e, int R, bool train) {
    const int L = d.L, C = d.dim[L], RT = R / 16;
    Lds lds{e.lds_bytes, {}};
    std::vector<std::string> names;
    for (int l = 0; l < L; ++l) { lds.add(nm("act", l), e.act_off[l], R * e.lda[l] * 2); names.push_back(nm("act", l)); }
    if (train)
        for (int l = 1; l <= L; ++l) { lds.add(nm("dlt", l), e.dlt_off[l], R * e.lda[l] * 2); names.push_back(nm("dlt", l)); }
    lds.add("logit", e.logit_off, R * FL_LOGIT_LD * 4);
    lds.add("cm", e.cm_off, FL_CM_INTS * 4);
    names.push_back("logit");
    names.push_back("cm");
    // lo parts: X's own buffer; hidden layers alias the delta buffers in the train layout
    lds.add("alo0", e.alo_off[0], R * e.lda[0] * 2);
    names.push_back("alo0");
    for (int l = 1; l < L; ++l) {
        if (train) CHECK(e.alo_off[l] == e.dlt_off[l], "train alo%d must alias dlt%d", l, l);
        else { lds.add(nm("alo", l), e.alo_off[l], R * e.lda[l] * 2); names.push_back(nm("alo", l)); }
    }
    lds.add("params", e.param_off, e.param_bytes);
    names.push_back("params");
    if (e.head_split > 1) {
        lds.add("part", e.part_off, e.head_split * R * C * 4);
        names.push_back("part");
    }
    lds.no_overlap(names);
    CHECK(e.lds_bytes <= FL_LDS_DYNAMIC_MAX, "LDS %d > %d", e.lds_bytes, FL_LDS_DYNAMIC_MAX);
    auto alo = [&](int l) { return (train && l >= 1) ? nm("dlt", l) : (l == 0 ? std::string("alo0") : nm("alo", l)); };
    // W images inside the parameter region, hi and lo
    for (int l = 0; l < L; ++l) {
        const int wb = fl_wrow(e.kp[l + 1], e.ldw[l], e.wgap);
        CHECK(e.w_off[l] >= e.param_off && e.w_off[l] + wb <= e.bias_off[0], "W%d hi outside the hi images", l);
        CHECK(e.w_off[l] + e.wlo_delta + wb <= e.param_off + e.param_bytes, "W%d lo outside params", l);
        CHECK(e.bias_off[l] + e.kp[l + 1] * 4 <= e.w_off[0] + e.wlo_delta, "b%d overlaps the lo images", l);
    }
    // staging: X hi / lo rows, all kp[0] columns
    for (int r = 0; r < R; ++r)
        for (int k = 0; k < e.kp[0]; ++k) {
            lds.touch("act0", e.act_off[0] + (r * e.lda[0] + k) * 2, 2);
            lds.touch("alo0", e.alo_off[0] + (r * e.lda[0] + k) * 2, 2);
        }
    // split-bf16 forward, every lane of every tile
    for (int l = 0; l < L; ++l) {
        const bool last = l + 1 == L;
        const int lda = e.lda[l], ksteps = e.kp[l] >> 5;
        const int ntiles = last ? (C + 15) >> 4 : e.kp[l + 1] >> 4;
        if (last && e.head_split > 1) {
            const int G = e.head_split, kper = (ksteps + G - 1) / G;
            for (int w = 0; w < G; ++w)
                for (int lane = 0; lane < 64; ++lane) {
                    const int lr = lane & 15, lg = lane >> 4, wc = fl_fwd_col(lr);
                    for (int ks = w * kper; ks < std::min(ksteps, w * kper + kper); ++ks) {
                        lds.touch("params", e.w_off[l] + fl_wbyte(e, l, wc, 32 * ks + 8 * lg), 16);
                        lds.touch("params", e.w_off[l] + e.wlo_delta + fl_wbyte(e, l, wc, 32 * ks + 8 * lg), 16);
                        for (int rt = 0; rt < RT; ++rt) {
                            lds.touch(nm("act", l), e.act_off[l] + (lr * lda + 8 * lg) * 2 + rt * 16 * lda * 2 + ks * 64, 16);
                            lds.touch(alo(l), e.alo_off[l] + (lr * lda + 8 * lg) * 2 + rt * 16 * lda * 2 + ks * 64, 16);
                        }
                    }
                    if (wc < C)
                        for (int rt = 0; rt < RT; ++rt)
                            for (int j = 0; j < 4; ++j)
                                lds.touch("part", e.part_off + ((w * R + rt * 16 + 4 * lg + j) * C + wc) * 4, 4);
                }
            for (int i = 0; i < R * C; ++i) lds.touch("logit", e.logit_off + ((i / C) * FL_LOGIT_LD + i % C) * 4, 4);
            continue;
        }
        for (int nt = 0; nt < ntiles; ++nt)
            for (int lane = 0; lane < 64; ++lane) {
                const int lr = lane & 15, lg = lane >> 4, n = nt * 16 + fl_fwd_col(lr);
                for (int ks = 0; ks < ksteps; ++ks) {
                    lds.touch("params", e.w_off[l] + fl_wbyte(e, l, n, 32 * ks + 8 * lg), 16);
                    lds.touch("params", e.w_off[l] + e.wlo_delta + fl_wbyte(e, l, n, 32 * ks + 8 * lg), 16);
                    for (int rt = 0; rt < RT; ++rt) {
                        lds.touch(nm("act", l), e.act_off[l] + (lr * lda + 8 * lg) * 2 + rt * 16 * lda * 2 + ks * 64, 16);
                        lds.touch(alo(l), e.alo_off[l] + (lr * lda + 8 * lg) * 2 + rt * 16 * lda * 2 + ks * 64, 16);
                    }
                }
                lds.touch("params", e.bias_off[l] + n * 4, 4);
                for (int rt = 0; rt < RT; ++rt)
                    for (int j = 0; j < 4; ++j) {
                        const int row = rt * 16 + fl_out_row(lg, j);
                        if (last) {
                            lds.touch("logit", e.logit_off + (row * FL_LOGIT_LD + n) * 4, 4);
                        } else {
                            lds.touch(nm("act", l + 1), e.act_off[l + 1] + (row * e.lda[l + 1] + n) * 2, 2);
                            lds.touch(alo(l + 1), e.alo_off[l + 1] + (row * e.lda[l + 1] + n) * 2, 2);
                        }
                    }
            }
    }
    if (!train) return;
    // backward: weight gradients (transposed reads of D_{l+1} and act_l) and input gradients
    for (int l = L - 1; l >= 0; --l) {
        const int K = d.dim[l], N = d.dim[l + 1], ldd = e.lda[l + 1], lda = e.lda[l];
        const int otiles = (N + 15) >> 4, itiles = (K + 15) >> 4;
        for (int t = 0; t < otiles * itiles; ++t)
            for (int lane = 0; lane < 64; ++lane) {
                const int ot = t / itiles, it = t - ot * itiles, lr = lane & 15, lg = lane >> 4, lq = lr >> 2, lp = lr & 3;
                if (RT >= 2) {
                    for (int h = 0; h < RT / 2; ++h) {
                        const int r0 = 32 * h + 4 * lg + lq;
                        for (int q = 0; q < 2; ++q) {
                            lds.touch(nm("dlt", l + 1), e.dlt_off[l + 1] + ((r0 + 16 * q) * ldd + ot * 16 + 4 * lp) * 2, 8);
                            lds.touch(nm("act", l), e.act_off[l] + ((r0 + 16 * q) * lda + it * 16 + 4 * lp) * 2, 8);
                        }
                    }
                } else {
                    const int r0 = 4 * lg + lq;
                    lds.touch(nm("dlt", l + 1), e.dlt_off[l + 1] + (r0 * ldd + ot * 16 + 4 * lp) * 2, 8);
                    lds.touch(nm("act", l), e.act_off[l] + (r0 * lda + it * 16 + 4 * lp) * 2, 8);
                }
            }
        if (l == 0) continue;
        const int it_tiles = e.kp[l] >> 4, osteps = e.kp[l + 1] >> 5;
        for (int it = 0; it < it_tiles; ++it)
            for (int lane = 0; lane < 64; ++lane) {
                const int lr = lane & 15, lg = lane >> 4, lq = lr >> 2, lp = lr & 3;
                for (int os = 0; os < osteps; ++os) {
                    for (int q = 0; q < 2; ++q)
                        lds.touch("params", e.w_off[l] + fl_wbyte(e, l, 32 * os + 8 * lg + lq + 4 * q, it * 16 + 4 * lp), 8);
                    for (int rt = 0; rt < RT; ++rt)
                        lds.touch(nm("dlt", l + 1), e.dlt_off[l + 1] + (lr * ldd + 8 * lg) * 2 + rt * 16 * ldd * 2 + os * 64, 16);
                }
                for (int rt = 0; rt < RT; ++rt)
                    for (int j = 0; j < 4; ++j) {
                        const int o = ((rt * 16 + fl_out_row(lg, j)) * lda + it * 16 + lr) * 2;
                        lds.touch(nm("act", l), e.act_off[l] + o, 2);
                        lds.touch(nm("dlt", l), e.dlt_off[l] + o, 2);
                    }
            }
    }
}

// Packed global image (Adam kernel, pack kernel, peer pack epilogue): every dense parameter's
// hi / lo / bias position stays inside [0, param_bytes).
static void check_packing(const MLPDesc& d, const MLPDescB& e) {
    std::vector<unsigned char> img((size_t)e.param_bytes);
    for (int di = 0; di < d.P; ++di) {
        int l = 0;
        while (l + 1 < d.L && di >= d.w_off[l + 1]) ++l;
        const int K = d.dim[l];
        if (di < d.b_off[l]) {
            const int q = di - d.w_off[l], n = q / K, k = q - n * K;
            const long pk = e.w_off[l] - e.param_off + fl_wbyte(e, l, n, k);
            CHECK(pk >= 0 && pk + e.wlo_delta + 2 <= e.param_bytes, "packed W%d (%d, %d) out of range", l, n, k);
            if (pk >= 0 && pk + e.wlo_delta + 2 <= e.param_bytes) { img[(size_t)pk] ^= 1; img[(size_t)(pk + e.wlo_delta)] ^= 1; }
        } else {
            const long pk = e.bias_off[l] - e.param_off + (di - d.b_off[l]) * 4;
            CHECK(pk >= 0 && pk + 4 <= e.w_off[0] - e.param_off + e.wlo_delta, "packed b%d out of range", l);
        }
    }
    // pack kernel items: 8 elements per item of every padded W row
    for (int l = 0; l < d.L; ++l)
        for (int n = 0; n < e.kp[l + 1]; ++n)
            for (int ch = 0; ch < (e.kp[l] >> 3); ++ch) {
                const long o = e.w_off[l] - e.param_off + fl_wbyte(e, l, n, 8 * ch);
                CHECK(o >= 0 && o + e.wlo_delta + 16 <= e.param_bytes, "pack item W%d row %d chunk %d", l, n, ch);
            }
}

static void check_fp32(const MLPDesc& d, int R) {
    const int L = d.L;
    CHECK(d.Pimg % 4 == 0, "Pimg %d not a multiple of 4", d.Pimg);
    for (int l = 0; l < L; ++l) {
        CHECK(d.ib_off[l] - d.iw_off[l] == fl_wrows(d.dim[l + 1]) * fl_ldw(d.dim[l]), "image W%d size", l);
        CHECK(d.ib_off[l] + ((d.dim[l + 1] + 15) & ~15) <= d.Pimg, "image b%d outside Pimg", l);
    }
    for (int l = 0; l <= L; ++l) CHECK(d.ld[l] % 8 == 4 && d.ld[l] >= d.dim[l], "ld[%d] = %d", l, d.ld[l]);
    CHECK(d.img_lds + d.Pimg == d.lds_floats, "image not at the LDS end");
    CHECK(d.act_off[L] + R * d.ld[L] <= d.cm_off, "activations overlap the counters");
}

// Register-resident scoring (fl_kernels_bf16.hip score_rows_regs): every forward phase of the
// training waves stays on waves [0, nw), and every global read of the scoring waves lies inside
// the packed parameter image (W rows < kp[l+1], k-blocks < kp[l] / 32, logits rows < 16,
// bias entries < kp[l+1]) and inside their register arrays (layer-0 input 1 k-block, the stored
// first hidden layer <= 2 k-blocks, <= 4 tiles).
static void check_lag_reg(const MLPDesc& d, const MLPDescB& e, int R) {
    const int L = d.L, C = d.dim[L], nw = FL_WAVES - FL_LAG_SPR * (R / 16);
    for (int l = 0; l + 1 < L; ++l)  // fwd_layer_bf16<RT, nw>: tile nt on wave nt % nw
        for (int nt = 0; nt < (e.kp[l + 1] >> 4); ++nt) CHECK(nt % nw < nw, "lag_reg: layer %d tile %d on a scoring wave", l, nt);
    CHECK(e.head_split <= nw && R * C <= nw * 64 && ((C + 15) >> 4) <= nw, "lag_reg: logits phase on a scoring wave");
    const int G = e.head_split;
    CHECK(C <= FL_LAG_MAX_C, "lag_reg: C %d", C);
    for (int j = 0; j < FL_LAG_SPR; ++j) {  // part ranges tile [0, G); upper waves' fit their LDS slots
        CHECK(fl_lag_w(G, j) <= fl_lag_w(G, j + 1), "lag_reg: part range %d of split %d", j, G);
        if (j > 0) CHECK(fl_lag_w(G, j + 1) - fl_lag_w(G, j) <= FL_LAG_PARTS, "lag_reg: parts of wave %d, split %d", j, G);
    }
    CHECK(fl_lag_w(G, 0) == 0 && fl_lag_w(G, FL_LAG_SPR) == G, "lag_reg: part ranges of split %d", G);
    CHECK(e.lds_bytes + fl_lag_reg_static_bytes(R) + 256 <= 160 * 1024, "lag_reg: LDS %d", e.lds_bytes);
    CHECK(L == 2 || L == 3, "lag_reg: %d layers", L);
    CHECK(e.kp[0] / 32 == 1, "lag_reg: input k-blocks %d", e.kp[0] / 32);
    if (L == 3) CHECK((e.kp[1] >> 4) <= 4 && (e.kp[1] >> 5) <= 2, "lag_reg: stored hidden layer %d", e.kp[1]);
    const int image = e.param_bytes;
    for (int l = 0; l < L; ++l) {
        const int rows = (l + 1 == L) ? 16 : e.kp[l + 1];
        CHECK(rows <= e.kp[l + 1], "lag_reg: layer %d rows", l);
        for (int n = 0; n < rows; ++n)
            for (int ks = 0; ks < (e.kp[l] >> 5); ++ks)
                for (int g = 0; g < 4; ++g) {
                    const int off = e.w_off[l] - e.param_off + fl_wrow(n, e.ldw[l], e.wgap) + 16 * (g ^ fl_wswz(n, e.wxor)) + ks * 64;
                    CHECK(off >= 0 && off + 16 + e.wlo_delta <= image && off % 16 == 0, "lag_reg: W%d read %d", l, off);
                }
        const int bend = e.bias_off[l] - e.param_off + ((rows + 15) & ~15) * 4;
        CHECK(bend <= image && (e.bias_off[l] - e.param_off) % 16 == 0, "lag_reg: bias %d", l);
    }
}

int main() {
    const std::vector<std::vector<int>> hidden = {{7}, {50, 200}, {33, 17, 9}, {100, 50}, {64, 64, 64}, {24, 12}};
    const int feats[] = {5, 14, 31, 33};
    const int classes[] = {2, 3, 10, 16};
    const int Rs[] = {16, 32, 64};
    int checked = 0, skipped = 0, lagreg = 0, levels[3] = {0, 0, 0};
    for (const auto& h : hidden)
        for (int F : feats)
            for (int C : classes)
                for (int R : Rs) {
                    std::vector<int> dims = {F};
                    dims.insert(dims.end(), h.begin(), h.end());
                    dims.push_back(C);
                    const int L = (int)dims.size() - 1;
                    if (L > FL_MAX_LAYERS) continue;
                    MLPDesc d;
                    fl_build_fp32_layout(dims.data(), L, R, &d);
                    if (R != 64 && (size_t)d.lds_floats * 4 <= FL_LDS_DYNAMIC_MAX) check_fp32(d, R);
                    MLPDescB e, ev;
                    fl_build_bf16_layout(d, R, &e, &ev);
                    if (std::max(e.lds_bytes, ev.lds_bytes) > FL_LDS_DYNAMIC_MAX) { ++skipped; continue; }  // engine refuses
                    check_bf16(d, e, R, true);
                    check_bf16(d, ev, R, false);
                    check_packing(d, e);
                    CHECK(e.head_split == ev.head_split, "train / eval logits split differ");
                    if (e.lag_reg) { check_lag_reg(d, e, R); ++lagreg; }
                    // operand reads: conflict free at level 2; level 1 leaves dgrad's transposed W
                    // reads 2-way (fl_common.h)
                    const BankStats bs = bank_conflicts_bf16(d, e, R);
                    if (e.level >= 1) {
                        CHECK(bs.act == 0 && bs.wfwd == 0, "dims %d-...-%d R %d level %d: act %ld / W fwd %ld extra LDS cycles",
                              F, C, R, e.level, bs.act, bs.wfwd);
                    }
                    if (e.level == 2) CHECK(bs.wdgrad == 0, "dims %d-...-%d R %d: W dgrad %ld extra LDS cycles", F, C, R, bs.wdgrad);
                    if (e.level >= 1) CHECK(bs.st == 0, "dims %d-...-%d R %d: stores %ld extra LDS cycles", F, C, R, bs.st);
                    ++levels[e.level];
                    ++checked;
                }
    std::printf("layouts checked: %d (bank levels 0/1/2: %d/%d/%d; skipped as too large for LDS: %d; register scoring: "
                "%d), failures: %d\n", checked, levels[0], levels[1], levels[2], skipped, lagreg, g_fail);
    // the flagship (BASELINE config 2) shape at R = 32
    {
        const int dims[] = {14, 50, 200, 2};
        MLPDesc d;
        fl_build_fp32_layout(dims, 3, 32, &d);
        MLPDescB e, ev;
        fl_build_bf16_layout(d, 32, &e, &ev);
        const BankStats bs = bank_conflicts_bf16(d, e, 32);
        std::printf("14-50-200-2 R 32: level %d, lds %d / %d bytes, head split %d, extra LDS cycles act %ld W fwd %ld "
                    "W dgrad %ld stores %ld\n", e.level, e.lds_bytes, ev.lds_bytes, e.head_split, bs.act, bs.wfwd, bs.wdgrad, bs.st);
        CHECK(e.level >= 1 && std::max(e.lds_bytes, ev.lds_bytes) <= (int)FL_LDS_DYNAMIC_MAX, "flagship layout");
        CHECK(e.lag_reg == 1, "flagship layout: lagged rounds score in registers");
    }
    return g_fail ? 1 : 0;
}
