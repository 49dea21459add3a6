// TEST INFRASTRUCTURE (tests/sanitize): drives the host-side C++ of librsac (csrc/rsac_host.hip)
// under ASan + UBSan and TSan.  Exit status 0 = every check passed (the sanitizers abort on a
// finding).  Checks, besides memory / UB / races:
//   1. scan_records (the device-listed scan replay) == scan_step on random rows, in rounds, with
//      LO stops and raised counts (the multi-GPU loop's usage);
//   2. mwc_subsets of 64 problems through parallel_for (16 threads) == the sequential draws;
//   3. the LM, EPnP and homography refits of 32 synthetic problems through parallel_for == the
//      same refits run sequentially (bitwise);
//   4. Rodrigues round trips;
//   5. the persistent parallel_for pool reused batch after batch, from two threads at once (the
//      second caller's batches run on its own thread while the pool is busy).
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <cmath>
#include <random>
#include <thread>
#include <vector>

#include "rsac_host.h"

using namespace rsac;

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                   \
        }                                                               \
    } while (0)

// the improvement records of rows [0, H) above floor0, as k_scan_rows lists them
static bool records(const int32_t *cnt, const int8_t *st, int64_t H, int floor0, std::vector<int32_t> &idx,
                    std::vector<int32_t> &rc, int32_t &first_neg) {
    idx.clear();
    rc.clear();
    first_neg = (int32_t)H;
    int f = floor0;
    for (int64_t i = 0; i < H; ++i) {
        if (st[i] < 0) {
            first_neg = (int32_t)i;
            break;
        }
        if (st[i] > 0 && cnt[i] > f) {
            idx.push_back((int32_t)i);
            rc.push_back(cnt[i]);
            f = cnt[i];
        }
    }
    return idx.size() <= 14;
}

static void check_scan(std::mt19937_64 &rng) {
    for (int trial = 0; trial < 400; ++trial) {
        const int64_t H = 1 + rng() % 4000;
        const int n = 500 + (int)(rng() % 5000);
        std::vector<int32_t> cnt(H);
        std::vector<int8_t> st(H);
        for (int64_t i = 0; i < H; ++i) {
            cnt[i] = (int32_t)(rng() % (uint64_t)n);
            st[i] = (rng() % 10) ? 1 : 0;
        }
        if (trial % 7 == 0) st[rng() % H] = -1;
        if (trial % 11 == 0)
            for (int64_t i = 0; i < std::min<int64_t>(H, 100); ++i) cnt[i] = (int32_t)(i * (n / 100));
        const bool lo = trial % 2;
        ScanState a, b;
        a.reset((int)H);
        b.reset((int)H);
        while (!b.done && b.iter < H) {
            const int64_t len = std::min<int64_t>(1 + rng() % 700, H - b.iter);
            CHECK(a.iter == b.iter);
            const int64_t p = b.iter;
            scan_step(b, cnt.data() + p, st.data() + p, len, n, 4, 0.995, lo);
            std::vector<int32_t> idx, rc;
            int32_t neg;
            const int floor0 = std::max(a.max_good, 3);
            if (records(cnt.data() + p, st.data() + p, len, floor0, idx, rc, neg))
                scan_records(a, idx.data(), rc.data(), (int)idx.size(), neg, len, n, 4, 0.995, lo);
            else
                scan_step(a, cnt.data() + p, st.data() + p, len, n, 4, 0.995, lo);
            CHECK(a.best == b.best && a.max_good == b.max_good && a.iter == b.iter && a.niters == b.niters &&
                  a.done == b.done && a.improved == b.improved);
            if (lo && b.improved) {  // a local optimisation raised the count (as rsac_scan_raise)
                const int raised = b.max_good + (int)(rng() % 3);
                for (ScanState *s : {&a, &b}) {
                    s->max_good = raised;
                    s->niters = update_num_iters(0.995, (double)(n - raised) / n, 4, (int)s->niters);
                    if (s->iter >= s->niters) s->done = true;
                    s->improved = false;
                }
            }
        }
    }
}

static void check_mwc(std::mt19937_64 &rng) {
    const int P = 64, Hs = 300;
    std::vector<int> ns(P);
    for (int p = 0; p < P; ++p) ns[p] = 4 + (int)(rng() % 400);
    std::vector<int32_t> par(P * Hs * 4), seq(P * Hs * 4);
    std::vector<int8_t> pst(P * Hs), sst(P * Hs);
    std::vector<Mwc> rngs(P);
    parallel_for(P, [&](int p) { mwc_subsets(rngs[p], ns[p], Hs, nullptr, &par[p * Hs * 4], &pst[p * Hs]); });
    for (int p = 0; p < P; ++p) {
        Mwc m;
        mwc_subsets(m, ns[p], Hs, nullptr, &seq[p * Hs * 4], &sst[p * Hs]);
    }
    CHECK(par == seq && pst == sst);
    // the draws against getSubset written with OpenCV's own remainder (rng.uniform = next() % n):
    // the sampler's direct-computation remainder must give the same subsets for any n
    for (int trial = 0; trial < 200; ++trial) {
        const int n = trial < 100 ? 4 + trial : 4 + (int)(rng() % 2000000);
        const int k = trial % 2 ? 5 : 4, H = 50;
        Mwc a, b;
        a.state = b.state = rng();
        std::vector<int32_t> got(H * k), want(H * k);
        std::vector<int8_t> st(H);
        mwc_subsets(a, n, H, nullptr, got.data(), st.data(), k);
        for (int h = 0; h < H; ++h)
            for (int i = 0; i < k; ++i) {
                int r;
                for (;;) {
                    r = b.uniform(0, n);
                    bool dup = false;
                    for (int j = 0; j < i; ++j) dup |= want[h * k + j] == r;
                    if (!dup) break;
                }
                want[h * k + i] = r;
            }
        CHECK(got == want);
        CHECK(a.state == b.state);
    }
}

struct Problem {
    std::vector<float> X, Y, Z, U, V, sx, sy, dx, dy;
    std::vector<uint8_t> mask;
    double cam[4];
    double R[9], t[3];
};

static Problem make_problem(std::mt19937_64 &rng, int n) {
    std::normal_distribution<double> g(0.0, 1.0);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    Problem pr;
    pr.cam[0] = 2000 + 500 * u(rng); pr.cam[1] = pr.cam[0]; pr.cam[2] = 1000; pr.cam[3] = 800;
    double r[3] = {0.3 * u(rng), 0.3 * u(rng), 0.3 * u(rng)};
    rodrigues_v2m(r, pr.R);
    pr.t[0] = 10 * u(rng); pr.t[1] = 10 * u(rng); pr.t[2] = 500 + 50 * u(rng);
    for (int i = 0; i < n; ++i) {
        const double X = 200 * u(rng), Y = 200 * u(rng), Z = 200 * u(rng);
        const double x = pr.R[0] * X + pr.R[1] * Y + pr.R[2] * Z + pr.t[0];
        const double y = pr.R[3] * X + pr.R[4] * Y + pr.R[5] * Z + pr.t[1];
        const double z = pr.R[6] * X + pr.R[7] * Y + pr.R[8] * Z + pr.t[2];
        const bool out = (rng() % 4) == 0;
        pr.X.push_back((float)X); pr.Y.push_back((float)Y); pr.Z.push_back((float)Z);
        pr.U.push_back((float)(out ? 2000 * (u(rng) + 1) : pr.cam[0] * x / z + pr.cam[2] + g(rng)));
        pr.V.push_back((float)(out ? 1600 * (u(rng) + 1) : pr.cam[1] * y / z + pr.cam[3] + g(rng)));
        pr.mask.push_back(out ? 0 : 1);
        // a homography pair: a plane seen from two views
        pr.sx.push_back((float)(X)); pr.sy.push_back((float)(Y));
        const double w = 0.0005 * X + 0.0003 * Y + 1.0;
        pr.dx.push_back((float)((1.1 * X + 0.1 * Y + 5) / w + (out ? 300 * u(rng) : 0.5 * g(rng))));
        pr.dy.push_back((float)((-0.05 * X + 0.9 * Y - 3) / w + (out ? 300 * u(rng) : 0.5 * g(rng))));
    }
    return pr;
}

struct Fit {
    double R[9], t[3], Re[9], te[3], H[9];
    int it;
    bool ep, hok;
};

static Fit fit(const Problem &p) {
    Fit f;
    memset(&f, 0, sizeof f);  // the padding too: the results are compared bytewise
    const int n = (int)p.X.size();
    double r0[3];
    rodrigues_m2v(p.R, r0);
    r0[0] += 0.01;
    rodrigues_v2m(r0, f.R);
    for (int k = 0; k < 3; ++k) f.t[k] = p.t[k] + 0.5;
    f.it = pnp_refine_lm(p.X.data(), p.Y.data(), p.Z.data(), p.U.data(), p.V.data(), p.mask.data(), n, p.cam, f.R,
                         f.t, 20);
    f.ep = pnp_epnp_host(p.X.data(), p.Y.data(), p.Z.data(), p.U.data(), p.V.data(), p.mask.data(), n, p.cam, f.Re,
                         f.te);
    f.hok = hom_refine(p.sx.data(), p.sy.data(), p.dx.data(), p.dy.data(), p.mask.data(), n, f.H);
    return f;
}

static void check_refits(std::mt19937_64 &rng) {
    const int P = 32;
    std::vector<Problem> probs;
    for (int p = 0; p < P; ++p) probs.push_back(make_problem(rng, 8 + (int)(rng() % 3000)));
    std::vector<Fit> par(P), seq(P);
    parallel_for(P, [&](int p) { par[p] = fit(probs[p]); });
    for (int p = 0; p < P; ++p) seq[p] = fit(probs[p]);
    for (int p = 0; p < P; ++p) {
        CHECK(memcmp(&par[p], &seq[p], sizeof(Fit)) == 0);
        double dR = 0;
        for (int k = 0; k < 9; ++k) dR = std::max(dR, std::fabs(seq[p].R[k] - probs[p].R[k]));
        CHECK(dR < 1e-2);
        CHECK(seq[p].ep && seq[p].hok);
    }
}

static void check_rodrigues(std::mt19937_64 &rng) {
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    for (int i = 0; i < 2000; ++i) {
        double r[3] = {u(rng), u(rng), u(rng)}, R[9], r2[3];
        const double s = 3.0 * std::fabs(u(rng)) / std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + 1e-30);
        for (double &v : r) v *= s;
        rodrigues_v2m(r, R);
        rodrigues_m2v(R, r2);
        const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        if (th > 1e-3 && th < 3.1)
            for (int k = 0; k < 3; ++k) CHECK(std::fabs(r2[k] - r[k]) < 1e-9);
    }
}

static void check_pool() {
    std::atomic<long> total{0};
    auto caller = [&](int salt) {
        for (int it = 0; it < 300; ++it) {
            const int P = 17 + (it * 7 + salt) % 150;
            std::vector<int> v(P, 0);
            parallel_for(P, [&](int p) { v[p] = p + 1; });
            long s = 0;
            for (int x : v) s += x;
            CHECK(s == (long)P * (P + 1) / 2);
            total += s;
        }
    };
    std::thread a(caller, 0), b(caller, 1);
    a.join();
    b.join();
    CHECK(total > 0);
}

int main() {
    std::mt19937_64 rng(20261017);
    check_pool();
    check_scan(rng);
    check_mwc(rng);
    check_refits(rng);
    check_rodrigues(rng);
    printf("host harness: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
