/* TEST INFRASTRUCTURE (tests/sanitize): drives the CPU restatement (oracle/rsac_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer: every whole loop (PnP with both samplers,
 * sequential and LO, homography, fundamental matrix), the refits, EPnP, the reprojection error
 * and the OpenMP hypothesis loop, on synthetic scenes with outliers, a 4-point minimum and a
 * degenerate (all identical) set.  Exit 0 = every check passed. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t orc_pnp_ransac(const float *, const float *, const float *, const float *, const float *, int, const double *,
                       double, double, int, uint64_t, int, double *, double *, uint8_t *, int32_t *, int64_t *);
int64_t orc_pnp_ransac_seq(const float *, const float *, const float *, const float *, const float *, int,
                           const double *, double, double, int, uint64_t, double *, double *, uint8_t *, int32_t *,
                           int64_t *);
int64_t orc_pnp_ransac_lo(const float *, const float *, const float *, const float *, const float *, int,
                          const double *, double, double, int, uint64_t, double *, double *, uint8_t *, int32_t *,
                          int64_t *, int32_t *);
void orc_pnp_hypotheses(const float *, const float *, const float *, const float *, const float *, int, const double *,
                        float, uint64_t, uint32_t, int64_t, int64_t, const int32_t *, const int8_t *, int32_t *,
                        int8_t *, double *);
void orc_pnp_hypotheses_mt(const float *, const float *, const float *, const float *, const float *, int,
                           const double *, float, uint64_t, int64_t, int64_t, int32_t *, int8_t *, int);
int orc_pnp_refine(const float *, const float *, const float *, const float *, const float *, const uint8_t *, int,
                   const double *, double *, double *, int);
int orc_pnp_epnp(const float *, const float *, const float *, const float *, const float *, const uint8_t *, int,
                 const double *, double *, double *);
int64_t orc_hom_ransac(const float *, const float *, const float *, const float *, int, double, double, int, uint64_t,
                       int, double *, uint8_t *, int32_t *, int64_t *);
int orc_hom_refine(const float *, const float *, const float *, const float *, const uint8_t *, int, double *);
int64_t orc_fm_ransac(const float *, const float *, const float *, const float *, int, double, double, int, uint64_t,
                      double *, uint8_t *, int32_t *, int64_t *);
double orc_reproj_mean_sum(const double *, const double *, const double *, const double *, const double *,
                           const uint8_t *, int, int *);
float orc_thr2(double);
void orc_rodrigues_v2m(const double *, double *);
int orc_cv_epnp(const float *, const float *, const float *, const float *, const float *, const int32_t *, int,
                const double *, double *, double *);
int64_t orc_pnp_ransac_k(const float *, const float *, const float *, const float *, const float *, int, const double *,
                         double, double, int, uint64_t, int, int, double *, double *, uint8_t *, int32_t *, int64_t *,
                         int);

static int g_fail = 0;
#define CHECK(c)                                                                          \
    do {                                                                                  \
        if (!(c)) {                                                                       \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            ++g_fail;                                                                     \
        }                                                                                 \
    } while (0)

static uint64_t g_rng = 88172645463325252ull;
static double urand(void) { /* xorshift64, in [0, 1) */
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) * (1.0 / 9007199254740992.0);
}

typedef struct {
    int n;
    float *X, *Y, *Z, *U, *V;
    double *p3, *p2;
    double cam[4];
} scene;

static scene make_scene(int n, double outl, int degenerate) {
    scene s;
    s.n = n;
    s.X = malloc(sizeof(float) * n); s.Y = malloc(sizeof(float) * n); s.Z = malloc(sizeof(float) * n);
    s.U = malloc(sizeof(float) * n); s.V = malloc(sizeof(float) * n);
    s.p3 = malloc(sizeof(double) * 3 * n); s.p2 = malloc(sizeof(double) * 2 * n);
    s.cam[0] = 2500; s.cam[1] = 2400; s.cam[2] = 1000; s.cam[3] = 800;
    double r[3] = {0.2, -0.1, 0.05}, R[9], t[3] = {3, -2, 800};
    orc_rodrigues_v2m(r, R);
    for (int i = 0; i < n; ++i) {
        double X = degenerate ? 1 : 300 * (urand() - 0.5), Y = degenerate ? 2 : 300 * (urand() - 0.5),
               Z = degenerate ? 3 : 300 * (urand() - 0.5);
        double x = R[0] * X + R[1] * Y + R[2] * Z + t[0], y = R[3] * X + R[4] * Y + R[5] * Z + t[1],
               z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        int out = urand() < outl;
        double u = out ? 2000 * urand() : s.cam[0] * x / z + s.cam[2] + urand() - 0.5;
        double v = out ? 1600 * urand() : s.cam[1] * y / z + s.cam[3] + urand() - 0.5;
        s.X[i] = (float)X; s.Y[i] = (float)Y; s.Z[i] = (float)Z; s.U[i] = (float)u; s.V[i] = (float)v;
        s.p3[3 * i] = X; s.p3[3 * i + 1] = Y; s.p3[3 * i + 2] = Z; s.p2[2 * i] = u; s.p2[2 * i + 1] = v;
    }
    return s;
}

static void free_scene(scene *s) {
    free(s->X); free(s->Y); free(s->Z); free(s->U); free(s->V); free(s->p3); free(s->p2);
}

static void pnp_checks(int n, double outl, int degenerate) {
    scene s = make_scene(n, outl, degenerate);
    double R[9], t[3], R2[9], t2[3];
    uint8_t *m = malloc(n), *m2 = malloc(n);
    int32_t good, good2, nlo;
    int64_t it, it2;
    for (int sampler = 0; sampler < 2; ++sampler) {
        int64_t b = orc_pnp_ransac(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, 8.0, 0.99, 2000, 7, sampler, R, t, m, &good, &it);
        if (degenerate) CHECK(b < 0);
        if (sampler == 0) {
            int64_t b2 = orc_pnp_ransac_seq(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, 8.0, 0.99, 2000, 7, R2, t2, m2, &good2,
                                            &it2);
            CHECK(b == b2 && good == good2 && it == it2 && memcmp(m, m2, n) == 0);
        }
        if (b >= 0) {
            memcpy(R2, R, sizeof R); memcpy(t2, t, sizeof t);
            orc_pnp_refine(s.X, s.Y, s.Z, s.U, s.V, m, n, s.cam, R2, t2, 20);
            orc_pnp_epnp(s.X, s.Y, s.Z, s.U, s.V, m, n, s.cam, R2, t2);
            int c = 0;
            double sum = orc_reproj_mean_sum(R, t, s.cam, s.p3, s.p2, m, n, &c);
            CHECK(c == good && isfinite(sum));
        }
    }
    /* OpenCV's default minimal solver (cv_epnp.c): EPnP-5 RANSAC on MWC subsets, and one
       degenerate (coincident) sample through JacobiSVD's zero-singular-value fill */
    orc_pnp_ransac_k(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, 8.0, 0.99, 500, 7, 1, 5, R, t, m, &good, &it, 1);
    {
        const int32_t dup[5] = {0, 0, 0, 0, 0};
        orc_cv_epnp(s.X, s.Y, s.Z, s.U, s.V, dup, 5, s.cam, R2, t2);
    }
    orc_pnp_ransac_lo(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, 8.0, 0.99, 2000, 7, R, t, m, &good, &it, &nlo);
    int32_t *c1 = malloc(sizeof(int32_t) * 600), *c2 = malloc(sizeof(int32_t) * 600);
    int8_t *s1 = malloc(600), *s2 = malloc(600);
    orc_pnp_hypotheses(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, orc_thr2(8.0), 3, 0, 11, 600, NULL, NULL, c1, s1, NULL);
    orc_pnp_hypotheses_mt(s.X, s.Y, s.Z, s.U, s.V, n, s.cam, orc_thr2(8.0), 3, 11, 600, c2, s2, 4);
    CHECK(memcmp(c1, c2, sizeof(int32_t) * 600) == 0 && memcmp(s1, s2, 600) == 0);
    free(c1); free(c2); free(s1); free(s2); free(m); free(m2);
    free_scene(&s);
}

static void hom_fm_checks(int n, double outl) {
    float *sx = malloc(sizeof(float) * n), *sy = malloc(sizeof(float) * n);
    float *dx = malloc(sizeof(float) * n), *dy = malloc(sizeof(float) * n);
    for (int i = 0; i < n; ++i) {
        double x = 500 * urand(), y = 500 * urand(), w = 0.0004 * x + 0.0002 * y + 1;
        int out = urand() < outl;
        sx[i] = (float)x; sy[i] = (float)y;
        dx[i] = (float)(out ? 800 * urand() : (1.1 * x + 0.05 * y + 7) / w + urand() - 0.5);
        dy[i] = (float)(out ? 800 * urand() : (-0.03 * x + 0.95 * y - 4) / w + urand() - 0.5);
    }
    double H[9], F[9];
    uint8_t *m = malloc(n);
    int32_t good;
    int64_t it;
    for (int sampler = 0; sampler < 2; ++sampler) {
        int64_t b = orc_hom_ransac(sx, sy, dx, dy, n, 3.0, 0.995, 2000, 5, sampler, H, m, &good, &it);
        if (b >= 0 && n > 4) orc_hom_refine(sx, sy, dx, dy, m, n, H);
    }
    if (n >= 8) orc_fm_ransac(sx, sy, dx, dy, n, 1.5, 0.99, 1500, 9, F, m, &good, &it);
    free(sx); free(sy); free(dx); free(dy); free(m);
}

int main(void) {
    pnp_checks(4, 0.0, 0);
    pnp_checks(12, 0.2, 0);
    pnp_checks(300, 0.5, 0);
    pnp_checks(5000, 0.5, 0);
    pnp_checks(50, 0.0, 1);
    hom_fm_checks(4, 0.0);
    hom_fm_checks(12, 0.3);
    hom_fm_checks(3000, 0.5);
    printf("oracle harness: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
