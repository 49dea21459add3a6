#include <algorithm>
// rsac_host.hip -- host-side sequential parts of the driver (see rsac_host.h).
#include "rsac_host.h"

#include <math.h>
#include <string.h>

#include <cfloat>
#include <memory>
#include <vector>

#include "rsac_math.h"

#include <pthread.h>

#include <condition_variable>
#include <mutex>

namespace rsac {

namespace {
// the persistent workers of parallel_for: nw threads wait for a batch (gen changes), take problem
// indices from next until P, and count themselves out in left; the caller takes indices too
struct HostPool {
    std::mutex mu;                 // held by the one batch in flight (try_lock: busy -> serial)
    std::mutex state;              // guards gen / fn / arg / P / nt / left and the condvars
    std::condition_variable go, done;
    uint64_t gen = 0;
    void (*fn)(void *, int) = nullptr;
    void *arg = nullptr;
    int P = 0, nt = 0, left = 0;
    std::atomic<int> next{0};
    int nw = 0;
    explicit HostPool(int workers) : nw(workers) {
        for (int w = 0; w < nw; ++w) std::thread([this, w] { loop(w); }).detach();
    }
    void loop(int w) {
        uint64_t seen = 0;
        for (;;) {
            void (*f)(void *, int);
            void *a;
            int n;
            {
                std::unique_lock<std::mutex> lk(state);
                go.wait(lk, [&] { return gen != seen; });
                seen = gen;
                if (w + 1 >= nt) continue;  // not one of this batch's nt - 1 workers
                f = fn;
                a = arg;
                n = P;
            }
            for (int p; (p = next.fetch_add(1)) < n;) f(a, p);
            std::lock_guard<std::mutex> lk(state);
            if (--left == 0) done.notify_one();
        }
    }
};
std::atomic<HostPool *> g_pool{nullptr};
std::mutex g_pool_mu;  // creation; held across fork (atfork), so the child finds it unlocked
int pool_threads() {
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::min(hw, 16);
}
void pool_prepare_fork() { g_pool_mu.lock(); }
void pool_parent_fork() { g_pool_mu.unlock(); }
void pool_child_fork() {  // the child has none of the workers: a new pool on demand
    g_pool.store(nullptr, std::memory_order_relaxed);
    g_pool_mu.unlock();
}
HostPool *pool() {
    HostPool *p = g_pool.load(std::memory_order_acquire);
    if (p) return p;
    static std::once_flag atfork_once;
    std::call_once(atfork_once, [] { pthread_atfork(pool_prepare_fork, pool_parent_fork, pool_child_fork); });
    std::lock_guard<std::mutex> lk(g_pool_mu);
    p = g_pool.load(std::memory_order_relaxed);
    if (!p) {
        p = new HostPool(pool_threads() - 1);  // never destroyed: the workers outlive main
        g_pool.store(p, std::memory_order_release);
    }
    return p;
}
}  // namespace

int host_pool_threads() { return pool_threads(); }

void host_pool_run(int P, int nt, void (*fn)(void *, int), void *arg) {
    HostPool *hp = pool();
    std::unique_lock<std::mutex> busy(hp->mu, std::try_to_lock);
    if (!busy.owns_lock()) {  // another batch holds the pool: this one on the calling thread
        for (int p = 0; p < P; ++p) fn(arg, p);
        return;
    }
    nt = std::min(nt, hp->nw + 1);
    {
        std::lock_guard<std::mutex> lk(hp->state);
        hp->fn = fn;
        hp->arg = arg;
        hp->P = P;
        hp->nt = nt;
        hp->left = nt - 1;
        hp->next.store(0);
        ++hp->gen;
    }
    hp->go.notify_all();
    for (int p; (p = hp->next.fetch_add(1)) < P;) fn(arg, p);
    std::unique_lock<std::mutex> lk(hp->state);
    hp->done.wait(lk, [&] { return hp->left == 0; });
}

void mwc_subsets(Mwc &rng, int n, int64_t H, const float *const *hom, int32_t *out, int8_t *status, int k) {
    // rng.uniform(0, n) = next() % n, the remainder by Lemire's direct computation (exact for
    // every 32-bit dividend and divisor; M = ceil(2^64 / n)) instead of a 32-bit division
    const uint64_t M = n > 0 ? UINT64_C(0xFFFFFFFFFFFFFFFF) / (uint32_t)n + 1 : 0;
    auto draw = [&]() -> int {
        const uint64_t lo = M * (uint64_t)rng.next();
        return (int)(((unsigned __int128)lo * (uint32_t)n) >> 64);
    };
    for (int64_t h = 0; h < H; ++h) {
        int32_t *idx = out + k * h;
        bool found = false;
        for (int att = 0; att < kMaxSubsetAttempts; ++att) {
            for (int i = 0; i < k; ++i) {
                int r;
                for (;;) {
                    r = draw();
                    bool dup = false;
                    for (int j = 0; j < i; ++j) dup |= (idx[j] == r);
                    if (!dup) break;
                }
                idx[i] = r;
            }
            if (hom) {
                float sx[4], sy[4], dx[4], dy[4];
                for (int j = 0; j < 4; ++j) {
                    sx[j] = hom[0][idx[j]]; sy[j] = hom[1][idx[j]];
                    dx[j] = hom[2][idx[j]]; dy[j] = hom[3][idx[j]];
                }
                if (!hom_check_subset(sx, sy, dx, dy)) continue;
            }
            found = true;
            break;
        }
        status[h] = found ? 1 : -1;
        if (!found) {
            for (int64_t g = h + 1; g < H; ++g) status[g] = -1;
            return;
        }
    }
}

int update_num_iters(double p, double ep, int model_points, int max_iters) {
    if (model_points <= 0) return -1;
    p = p > 0. ? p : 0.; p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
    double num = 1. - p;
    if (num < DBL_MIN) num = DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)lrint(num / denom);
}

// update_num_iters(p, (n - c) / n, model_points, max_iters) with its pow and logs (~47 ns) kept in
// a per-thread direct-mapped table keyed by (p, n, c, model_points): the same num and denom, so
// the same result; the scan replays of a batched call (C3: ~1500 updates over 1024 problems of
// equal size) see few distinct counts
int update_num_iters_count(double p, int n, int c, int model_points, int max_iters) {
    struct Entry {
        double p = -1.0, num = 0.0, denom = 0.0;
        int n = -1, c = -1, mp = -1;
        bool zero = false;  // denom < DBL_MIN: the result is 0
    };
    static thread_local Entry table[1024];
    if (model_points <= 0) return -1;
    Entry &e = table[((unsigned)c * 2654435761u ^ (unsigned)n * 40503u ^ (unsigned)model_points) & 1023u];
    if (!(e.p == p && e.n == n && e.c == c && e.mp == model_points)) {
        double pc = p > 0. ? p : 0.; pc = pc < 1. ? pc : 1.;
        double ep = (double)(n - c) / n;
        ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
        double num = 1. - pc;
        if (num < DBL_MIN) num = DBL_MIN;
        double denom = 1. - pow(1. - ep, model_points);
        e.p = p; e.n = n; e.c = c; e.mp = model_points;
        e.zero = denom < DBL_MIN;
        if (!e.zero) {
            e.num = log(num);
            e.denom = log(denom);
        }
    }
    if (e.zero) return 0;
    return (e.denom >= 0 || -e.num >= max_iters * (-e.denom)) ? max_iters : (int)lrint(e.num / e.denom);
}

void scan_step(ScanState &s, const int32_t *counts, const int8_t *status, int64_t count, int n, int model_points,
               double confidence, bool stop_on_improve) {
    if (s.done) return;
    const int64_t begin = s.iter;
    int64_t i = begin;
    for (; i < begin + count; ++i) {
        if (i >= s.niters) break;
        const int8_t st = status[i - begin];
        if (st < 0) { s.done = true; break; }
        if (st == 0) continue;
        const int32_t c = counts[i - begin];
        const int32_t floor_c = s.max_good > model_points - 1 ? s.max_good : model_points - 1;
        if (c > floor_c) {
            s.best = i;
            s.max_good = c;
            s.niters = update_num_iters_count(confidence, n, c, model_points, (int)s.niters);
            if (stop_on_improve) {
                s.improved = true;
                ++i;
                break;
            }
        }
    }
    s.iter = i;
    if (i >= s.niters) s.done = true;
}

void scan_records(ScanState &s, const int32_t *idx, const int32_t *cnt, int nrec, int32_t first_neg, int64_t H, int n,
                  int model_points, double confidence, bool stop_on_improve) {
    // scan_step over the round [s.iter, s.iter + H) replayed on its records: idx / first_neg are
    // relative to the round's start and the records are the strict prefix maxima above the
    // scan's floor, so between records nothing changes.  scan_step stops at the first index i
    // >= niters (niters only shrinks; after an improvement at p the next index checked is p + 1,
    // so the scan ends at max(p + 1, niters)) or at a status < 0 (first_neg).
    const int64_t begin = s.iter, end = begin + H, neg = begin + first_neg;
    int64_t cur = begin;  // the next index the sequential scan would check
    s.improved = false;
    for (int r = 0; r < nrec; ++r) {
        const int64_t pos = begin + idx[r];
        if (pos >= std::min<int64_t>(neg, s.niters)) break;
        if (cnt[r] <= std::max(s.max_good, model_points - 1)) continue;  // below a raised floor (LO)
        s.best = pos;
        s.max_good = cnt[r];
        s.niters = update_num_iters_count(confidence, n, cnt[r], model_points, (int)s.niters);
        cur = pos + 1;
        if (stop_on_improve) {
            s.improved = true;
            s.iter = cur;
            if (cur >= s.niters) s.done = true;
            return;
        }
    }
    const int64_t stop = std::min<int64_t>(std::max<int64_t>(cur, s.niters), neg);
    if (stop < end) {
        s.iter = stop;
        s.done = true;
    } else {
        s.iter = end;
        s.done = end >= s.niters;
    }
}

// cv::Rodrigues on the host: the deterministic forms of rsac_math.h (the device's and the
// oracle's bits)
void rodrigues_v2m(const double r[3], double R[9]) { rodrigues_v2m_det(r, R); }
void rodrigues_m2v(const double R[9], double r[3]) { rodrigues_m2v_det(R, r); }

namespace {

// host reducer of pnp_lm_refine: the GPU kernel's summation order (rsac_math.h)
struct HostLmReducer {
    const float *X, *Y, *Z, *U, *V;
    const uint8_t *mask;
    int n;
    Cam k;
    double c[3];  // centre of the refit frame
    std::vector<double> part = std::vector<double>((size_t)lm_blocks(n) * kLmThreads * kLmTerms);
    double accs[2][kLmTerms] = {};
    double *acc_buf(int k) { return accs[k]; }
    void mark(int) {}
    void normal(const double *R, const double *t, double *acc) {
        lm_reduce_blocks_host(n, mask, kLmTerms, part.data(), acc, [&](int i, double *a) {
            pnp_lm_point(R, t, k, (double)X[i] - c[0], (double)Y[i] - c[1], (double)Z[i] - c[2], (double)U[i],
                         (double)V[i], a);
        });
    }
    double cost(const double *R, const double *t) {
        double s;
        lm_reduce_blocks_host(n, mask, 1, part.data(), &s, [&](int i, double *a) {
            a[0] += pnp_lm_cost_point(R, t, k, (double)X[i] - c[0], (double)Y[i] - c[1], (double)Z[i] - c[2],
                                      (double)U[i], (double)V[i]);
        });
        return s;
    }
};

struct HostEpnpReducer {
    const float *X, *Y, *Z, *U, *V;
    const uint8_t *mask;
    int n;
    double c[3];
    std::vector<double> part = std::vector<double>((size_t)kLmThreads * kRedMax);
    template <int NV, class F>
    void sum(F f, double *out) {
        lm_reduce_host(n, mask, NV, part.data(), out, [&](int i, double *a) {
            f((double)X[i] - c[0], (double)Y[i] - c[1], (double)Z[i] - c[2], (double)U[i], (double)V[i], a);
        });
    }
    bool first(double *p) {
        for (int i = 0; i < n; ++i)
            if (mask[i]) {
                p[0] = (double)X[i] - c[0];
                p[1] = (double)Y[i] - c[1];
                p[2] = (double)Z[i] - c[2];
                return true;
            }
        return false;
    }
};

}  // namespace

bool pnp_epnp_host(const float *X, const float *Y, const float *Z, const float *U, const float *V, const uint8_t *mask,
                   int n, const double cam[4], double R[9], double t[3]) {
    if (n <= 0) return false;
    auto red = std::make_unique<HostEpnpReducer>();
    *red = HostEpnpReducer{X, Y, Z, U, V, mask, n, {(double)X[0], (double)Y[0], (double)Z[0]}};
    double Rn[9], tn[3];
    if (!pnp_epnp(*red, Cam{cam[0], cam[1], cam[2], cam[3]}, Rn, tn)) return false;
    lm_from_centred(Rn, red->c, tn);
    for (int j = 0; j < 9; ++j) R[j] = Rn[j];
    for (int j = 0; j < 3; ++j) t[j] = tn[j];
    return true;
}

int pnp_refine_lm(const float *X, const float *Y, const float *Z, const float *U, const float *V, const uint8_t *mask,
                  int n, const double cam[4], double R[9], double t[3], int max_iter) {
    if (n <= 0) return 0;
    HostLmReducer red{X, Y, Z, U, V, mask, n, Cam{cam[0], cam[1], cam[2], cam[3]}, {(double)X[0], (double)Y[0], (double)Z[0]}};
    lm_to_centred(R, red.c, t);
    const int it = pnp_lm_refine(red, R, t, max_iter);
    lm_from_centred(R, red.c, t);
    return it;
}

// Symmetric eigen-decomposition by cyclic Jacobi (cv::eigen's method): A (n x n,
// destroyed) -> eigenvalues on the diagonal, eigenvectors in the columns of V.
// Stops when the off-diagonal mass is below 1e-32 of the matrix's.
static void jacobi_sym(int n, double *A, double *V) {
    double frob = 0;
    for (int i = 0; i < n * n; ++i) frob += A[i] * A[i];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
        if (off <= 1e-32 * frob || off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                const double app = A[p * n + p], aqq = A[q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

static void jacobi_min_evec(int n, double *A, double *v_out) {
    double V[81];
    jacobi_sym(n, A, V);
    int mi = 0;
    for (int i = 1; i < n; ++i)
        if (A[i * n + i] < A[mi * n + mi]) mi = i;
    for (int k = 0; k < n; ++k) v_out[k] = V[k * n + mi];
}

// Residuals of HomographyRefineCallback::compute (OpenCV fundam.cpp) over the
// inliers: projection - dst (x, y interleaved); Jacobian w.r.t. h0..h7 (h8 = 1).
static void hom_residuals(const double *h, const float *sx, const float *sy, const float *dx, const float *dy,
                          const uint8_t *mask, int n, double *r, double *J) {
    int q = 0;
    for (int i = 0; i < n; ++i) {
        if (!mask[i]) continue;
        const double Mx = sx[i], My = sy[i];
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        r[2 * q] = xi - dx[i];
        r[2 * q + 1] = yi - dy[i];
        if (J) {
            double *jx = J + 16 * q, *jy = jx + 8;
            jx[0] = Mx * ww; jx[1] = My * ww; jx[2] = ww; jx[3] = jx[4] = jx[5] = 0.;
            jx[6] = -Mx * ww * xi; jx[7] = -My * ww * xi;
            jy[0] = jy[1] = jy[2] = 0.; jy[3] = Mx * ww; jy[4] = My * ww; jy[5] = ww;
            jy[6] = -Mx * ww * yi; jy[7] = -My * ww * yi;
        }
        ++q;
    }
}

// A = J^T J, v = J^T r for m residuals and 8 parameters
static void normal_eqs(const double *J, const double *r, int m, double *A, double *v) {
    std::fill(A, A + 64, 0.0);
    std::fill(v, v + 8, 0.0);
    for (int k = 0; k < m; ++k) {
        const double *jr = J + 8 * k;
        for (int a = 0; a < 8; ++a) {
            v[a] += jr[a] * r[k];
            for (int b = 0; b < 8; ++b) A[a * 8 + b] += jr[a] * jr[b];
        }
    }
}

// 8x8 symmetric A -> eigenvalues W (diagonal), vectors V; |w| <= 8 eps max|w|
// zeroed, as cv::solve / cv::invert with DECOMP_EIG drop them
static void eig8(const double *A, double *W, double *V) {
    std::copy(A, A + 64, W);
    jacobi_sym(8, W, V);
    double wmax = 0;
    for (int i = 0; i < 8; ++i) wmax = fmax(wmax, fabs(W[i * 8 + i]));
    const double tol = wmax * 8 * DBL_EPSILON;
    for (int i = 0; i < 8; ++i)
        if (fabs(W[i * 8 + i]) <= tol) W[i * 8 + i] = 0;
}

// x = A^+ b (cv::solve DECOMP_EIG)
static void solve_eig8(const double *A, const double *b, double *x) {
    double W[64], V[64];
    eig8(A, W, V);
    std::fill(x, x + 8, 0.0);
    for (int e = 0; e < 8; ++e) {
        const double w = W[e * 8 + e];
        if (w == 0) continue;
        double c = 0;
        for (int k = 0; k < 8; ++k) c += V[k * 8 + e] * b[k];
        c /= w;
        for (int k = 0; k < 8; ++k) x[k] += c * V[k * 8 + e];
    }
}

// max_a |(A^+)_aa| (cv::invert DECOMP_EIG, diagonal only)
static double max_diag_pinv(const double *A) {
    double W[64], V[64], maxval = DBL_EPSILON;
    eig8(A, W, V);
    for (int a = 0; a < 8; ++a) {
        double d = 0;
        for (int e = 0; e < 8; ++e)
            if (W[e * 8 + e] != 0) d += V[a * 8 + e] * V[a * 8 + e] / W[e * 8 + e];
        maxval = fmax(maxval, fabs(d));
    }
    return maxval;
}

// cv::LMSolver::run of OpenCV 4.x (levmarq.cpp, LMSolverImpl) on h0..h7:
// damping lambda * diag(J^T J at the start), gain-ratio schedule (0.25 / 0.75),
// lambda -> 0 below lc and restart from 1 / max diag(A^-1), at most max_iters
// iterations, stop when |d|inf or |r|inf < FLT_EPSILON.
static int hom_lm(const float *sx, const float *sy, const float *dx, const float *dy, const uint8_t *mask, int n,
                  double H[9], int max_iters) {
    int m = 0;
    for (int i = 0; i < n; ++i) m += mask[i] != 0;
    if (m == 0) return 0;
    m *= 2;
    std::vector<double> r(m), rd(m), J((size_t)m * 8);
    double x[9], xd[9], A[64], Ap[64], v[8], D[8], d[8];
    std::copy(H, H + 9, x);
    std::copy(H, H + 9, xd);
    hom_residuals(x, sx, sy, dx, dy, mask, n, r.data(), J.data());
    double S = 0;
    for (int k = 0; k < m; ++k) S += r[k] * r[k];
    normal_eqs(J.data(), r.data(), m, A, v);
    for (int a = 0; a < 8; ++a) D[a] = A[a * 8 + a];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        std::copy(A, A + 64, Ap);
        for (int a = 0; a < 8; ++a) Ap[a * 8 + a] += lambda * D[a];
        solve_eig8(Ap, v, d);
        for (int a = 0; a < 8; ++a) xd[a] = x[a] - d[a];
        hom_residuals(xd, sx, sy, dx, dy, mask, n, rd.data(), nullptr);
        double Sd = 0;
        for (int k = 0; k < m; ++k) Sd += rd[k] * rd[k];
        double dS = 0;  // d . (2 v - A d)
        for (int a = 0; a < 8; ++a) {
            double ad = 0;
            for (int b = 0; b < 8; ++b) ad += A[a * 8 + b] * d[b];
            dS += d[a] * (2 * v[a] - ad);
        }
        const double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int a = 0; a < 8; ++a) t += d[a] * v[a];
            double nu = (Sd - S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = fmin(fmax(nu, 2.), 10.);
            if (lambda == 0) {
                const double maxval = max_diag_pinv(A);
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            std::copy(xd, xd + 8, x);
            hom_residuals(x, sx, sy, dx, dy, mask, n, r.data(), J.data());
            normal_eqs(J.data(), r.data(), m, A, v);
        }
        iter++;
        double dinf = 0, rinf = 0;
        for (int a = 0; a < 8; ++a) dinf = fmax(dinf, fabs(d[a]));
        for (int k = 0; k < m; ++k) rinf = fmax(rinf, fabs(r[k]));
        if (!(iter < max_iters && dinf >= FLT_EPSILON && rinf >= FLT_EPSILON)) break;
    }
    std::copy(x, x + 8, H);
    H[8] = 1.0;
    return iter;
}

bool hom_refine(const float *sx, const float *sy, const float *dx, const float *dy, const uint8_t *mask, int n,
                double H[9]) {
    std::vector<int32_t> idx;
    for (int i = 0; i < n; ++i)
        if (mask[i]) idx.push_back(i);
    const int m = (int)idx.size();
    if (m < 4) return false;
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < m; ++i) {
        int p = idx[i];
        cmx += dx[p]; cmy += dy[p]; cMx += sx[p]; cMy += sy[p];
    }
    cmx /= m; cmy /= m; cMx /= m; cMy /= m;
    for (int i = 0; i < m; ++i) {
        int p = idx[i];
        smx += fabs(dx[p] - cmx); smy += fabs(dy[p] - cmy);
        sMx += fabs(sx[p] - cMx); sMy += fabs(sy[p] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return false;
    smx = m / smx; smy = m / smy; sMx = m / sMx; sMy = m / sMy;
    double LtL[81] = {0};
    for (int i = 0; i < m; ++i) {
        int p = idx[i];
        double x = (dx[p] - cmx) * smx, y = (dy[p] - cmy) * smy;
        double X = (sx[p] - cMx) * sMx, Y = (sy[p] - cMy) * sMy;
        double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) LtL[j * 9 + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < j; ++k) LtL[j * 9 + k] = LtL[k * 9 + j];
    double hv[9];
    jacobi_min_evec(9, LtL, hv);
    double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9], H0[9];
    mat3mul(invHnorm, hv, T);
    mat3mul(T, Hnorm2, H0);
    double sc = 1. / H0[8];
    for (int k = 0; k < 9; ++k) H[k] = H0[k] * sc;
    hom_lm(sx, sy, dx, dy, mask, n, H, 10);
    return true;
}

}  // namespace rsac
