// The scikit-learn epoch shuffles of the MLPClassifier minibatch loop, generated natively.
//
// sklearn's _fit_stochastic draws `sample_idx = shuffle(sample_idx, random_state=rs)` once per
// epoch (fedmi/models/sklearn_mlp.py epoch_permutations); with a legacy numpy RandomState that is
// rs.shuffle(arange(n)) -- a Fisher-Yates pass drawing random_interval(i) for i = n-1 .. 1 from the
// MT19937 stream -- composed with the previous epoch's order.  The float64 estimator pre-computes
// every epoch's order for its device loop; in Python that took ~94 ms per 400-epoch fit of 8000 rows
// (profiles/h_sweep_phases_r6.log: most of the [H] sweep's job preparation).  This is the same
// generator (numpy's mt19937.c and random_interval, state in / state out), so the orders and the
// RandomState's state afterwards are numpy's bit for bit (tests/test_sklearn_estimator.py).
#include <cstddef>
#include <cstdint>
#include <vector>

namespace {
constexpr int MT_N = 624, MT_M = 397;

struct Mt19937 {
    uint32_t key[MT_N];
    uint32_t out[MT_N];   // the tempered outputs of the current block (filled by gen(): one vectorisable pass)
    int pos;

    void gen() {
        constexpr uint32_t A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
        int i = 0;
        uint32_t y;
        for (; i < MT_N - MT_M; ++i) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + MT_M] ^ (y >> 1) ^ (-(y & 1u) & A);
        }
        for (; i < MT_N - 1; ++i) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1u) & A);
        }
        y = (key[MT_N - 1] & UPPER) | (key[0] & LOWER);
        key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ (-(y & 1u) & A);
        pos = 0;
        temper_all();
    }
    void temper_all() {
        for (int i = 0; i < MT_N; ++i) {
            uint32_t y = key[i];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            out[i] = y;
        }
    }
    uint32_t next32() {
        if (pos == MT_N) gen();
        return out[pos++];
    }
};
}  // namespace

// perms [epochs][n]: epoch e's sample order; key / pos: the MT19937 state in (numpy get_state) and
// out (for set_state).  n < 2^31.
void sk_epoch_perms(uint32_t* key, int* pos, int n, int epochs, int32_t* perms) {
    Mt19937 mt;
    for (int i = 0; i < MT_N; ++i) mt.key[i] = key[i];
    mt.pos = *pos;
    mt.temper_all();   // (the block numpy is in the middle of: positions pos.. are still to be drawn)
    std::vector<int32_t> idx(n), ind(n), nxt(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    for (int e = 0; e < epochs; ++e) {
        for (int i = 0; i < n; ++i) ind[i] = i;
        // random_interval(i)'s mask (the smallest 2^k - 1 >= i) only shrinks as i falls: kept, not
        // recomputed per draw (the same values: masked rejection sampling either way)
        uint32_t mask = (uint32_t)(n - 1);
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        for (int i = n - 1; i >= 1; --i) {
            if ((uint32_t)i <= (mask >> 1)) mask >>= 1;
            uint32_t j;
            while ((j = (mt.next32() & mask)) > (uint32_t)i) {
            }
            const int32_t t = ind[i];
            ind[i] = ind[j];
            ind[j] = t;
        }
        for (int i = 0; i < n; ++i) nxt[i] = idx[ind[i]];
        idx.swap(nxt);
        for (int i = 0; i < n; ++i) perms[(std::size_t)e * n + i] = idx[i];
    }
    for (int i = 0; i < MT_N; ++i) key[i] = mt.key[i];
    *pos = mt.pos;
}
