// rsac_geo.h -- UTM <-> WGS84 and the DEM ray march of the reference's
// pixel -> ground-point path (main_v1.py:547-573 pixel_to_ray, :635-656
// ray_intersect_dem, :36-57 GeoCoordTransformer on EPSG:32650).
//
// The reference calls pyproj (EPSG:4326 <-> EPSG:32650) and scipy's
// RegularGridInterpolator.  pyproj is not installed here, so the projection is
// restated from its published algorithm: the transverse Mercator series of
// Krueger to sixth order in n (Karney, "Transverse Mercator with an accuracy of
// a few nanometers", J. Geodesy 2011), which is what PROJ's default UTM
// ("etmerc"/Poder-Engsager) implements; accuracy ~nm within the zone.  Series
// are summed with Clenshaw recurrences on the complex argument (Karney §4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rsac_math.h"

namespace rsac {

struct UtmZone {
    double lon0;  // central meridian, radians
    double fn;    // false northing (0 N, 1e7 S)
};

// WGS84 and the UTM scale
constexpr double kWgsA = 6378137.0;
constexpr double kWgsF = 1.0 / 298.257223563;
constexpr double kUtmK0 = 0.9996;
constexpr double kUtmFE = 500000.0;

struct TmConst {
    double n, e, A;      // third flattening, eccentricity, rectifying radius
    double alpha[6];     // forward series
    double beta[6];      // inverse series
    double delta[6];     // conformal -> geodetic latitude
};

RSAC_HD TmConst tm_const() {
    const double f = kWgsF;
    const double n = f / (2.0 - f);
    const double n2 = n * n, n3 = n2 * n, n4 = n3 * n, n5 = n4 * n, n6 = n5 * n;
    TmConst c;
    c.n = n;
    c.e = dsqrt(f * (2.0 - f));
    c.A = kWgsA / (1.0 + n) * (1.0 + n2 / 4.0 + n4 / 64.0 + n6 / 256.0);
    c.alpha[0] = n / 2.0 - 2.0 * n2 / 3.0 + 5.0 * n3 / 16.0 + 41.0 * n4 / 180.0 - 127.0 * n5 / 288.0 +
                 7891.0 * n6 / 37800.0;
    c.alpha[1] = 13.0 * n2 / 48.0 - 3.0 * n3 / 5.0 + 557.0 * n4 / 1440.0 + 281.0 * n5 / 630.0 -
                 1983433.0 * n6 / 1935360.0;
    c.alpha[2] = 61.0 * n3 / 240.0 - 103.0 * n4 / 140.0 + 15061.0 * n5 / 26880.0 + 167603.0 * n6 / 181440.0;
    c.alpha[3] = 49561.0 * n4 / 161280.0 - 179.0 * n5 / 168.0 + 6601661.0 * n6 / 7257600.0;
    c.alpha[4] = 34729.0 * n5 / 80640.0 - 3418889.0 * n6 / 1995840.0;
    c.alpha[5] = 212378941.0 * n6 / 319334400.0;
    c.beta[0] = n / 2.0 - 2.0 * n2 / 3.0 + 37.0 * n3 / 96.0 - n4 / 360.0 - 81.0 * n5 / 512.0 + 96199.0 * n6 / 604800.0;
    c.beta[1] = n2 / 48.0 + n3 / 15.0 - 437.0 * n4 / 1440.0 + 46.0 * n5 / 105.0 - 1118711.0 * n6 / 3870720.0;
    c.beta[2] = 17.0 * n3 / 480.0 - 37.0 * n4 / 840.0 - 209.0 * n5 / 4480.0 + 5569.0 * n6 / 90720.0;
    c.beta[3] = 4397.0 * n4 / 161280.0 - 11.0 * n5 / 504.0 - 830251.0 * n6 / 7257600.0;
    c.beta[4] = 4583.0 * n5 / 161280.0 - 108847.0 * n6 / 3991680.0;
    c.beta[5] = 20648693.0 * n6 / 638668800.0;
    c.delta[0] = 2.0 * n - 2.0 * n2 / 3.0 - 2.0 * n3 + 116.0 * n4 / 45.0 + 26.0 * n5 / 45.0 - 2854.0 * n6 / 675.0;
    c.delta[1] = 7.0 * n2 / 3.0 - 8.0 * n3 / 5.0 - 227.0 * n4 / 45.0 + 2704.0 * n5 / 315.0 + 2323.0 * n6 / 945.0;
    c.delta[2] = 56.0 * n3 / 15.0 - 136.0 * n4 / 35.0 - 1262.0 * n5 / 105.0 + 73814.0 * n6 / 2835.0;
    c.delta[3] = 4279.0 * n4 / 630.0 - 332.0 * n5 / 35.0 - 399572.0 * n6 / 14175.0;
    c.delta[4] = 4174.0 * n5 / 315.0 - 144838.0 * n6 / 6237.0;
    c.delta[5] = 601676.0 * n6 / 22275.0;
    return c;
}

RSAC_HD UtmZone utm_zone(int zone, bool south) {
    const double kPi = 3.14159265358979323846;
    return UtmZone{(-183.0 + 6.0 * zone) * kPi / 180.0, south ? 10000000.0 : 0.0};
}

// S = sum_{j=1..6} c_j sin(2 j zeta) for complex zeta = (xr, xi), by Clenshaw
RSAC_HD void clenshaw_sin_c(const double *c, double xr, double xi, double &sr, double &si) {
    const double s2 = sin(2.0 * xr), c2 = cos(2.0 * xr), sh2 = sinh(2.0 * xi), ch2 = cosh(2.0 * xi);
    // a = 2 cos(2 zeta)
    const double ar = 2.0 * c2 * ch2, ai = -2.0 * s2 * sh2;
    double y1r = 0.0, y1i = 0.0, y2r = 0.0, y2i = 0.0;
    for (int j = 5; j >= 0; --j) {
        const double yr = ar * y1r - ai * y1i - y2r + c[j];
        const double yi = ar * y1i + ai * y1r - y2i;
        y2r = y1r; y2i = y1i;
        y1r = yr; y1i = yi;
    }
    // S = y1 sin(2 zeta), sin(2 zeta) = (s2 ch2, c2 sh2)
    const double br = s2 * ch2, bi = c2 * sh2;
    sr = y1r * br - y1i * bi;
    si = y1r * bi + y1i * br;
}

// S = sum_{j=1..6} c_j sin(2 j x), real Clenshaw
RSAC_HD double clenshaw_sin(const double *c, double x) {
    const double a = 2.0 * cos(2.0 * x);
    double y1 = 0.0, y2 = 0.0;
    for (int j = 5; j >= 0; --j) {
        const double y = a * y1 - y2 + c[j];
        y2 = y1;
        y1 = y;
    }
    return y1 * sin(2.0 * x);
}

// easting, northing -> lon, lat (degrees); EPSG:326zz / 327zz inverse
RSAC_HD void utm_inverse(const TmConst &k, const UtmZone &z, double E, double N, double &lon, double &lat) {
    const double kDeg = 57.29577951308232;
    const double xi = (N - z.fn) / (kUtmK0 * k.A);
    const double eta = (E - kUtmFE) / (kUtmK0 * k.A);
    double sr, si;
    clenshaw_sin_c(k.beta, xi, eta, sr, si);
    const double xip = xi - sr, etap = eta - si;
    const double chi = asin(sin(xip) / cosh(etap));
    lat = (chi + clenshaw_sin(k.delta, chi)) * kDeg;
    lon = (z.lon0 + atan2(sinh(etap), cos(xip))) * kDeg;
}

// lon, lat (degrees) -> easting, northing; EPSG:326zz / 327zz forward
RSAC_HD void utm_forward(const TmConst &k, const UtmZone &z, double lon, double lat, double &E, double &N) {
    const double kRad = 0.017453292519943295;
    const double phi = lat * kRad, dl = lon * kRad - z.lon0;
    const double sp = sin(phi);
    const double t = sinh(atanh(sp) - k.e * atanh(k.e * sp));
    const double xip = atan2(t, cos(dl));
    const double etap = atanh(sin(dl) / dsqrt(1.0 + t * t));
    double sr, si;
    clenshaw_sin_c(k.alpha, xip, etap, sr, si);
    N = z.fn + kUtmK0 * k.A * (xip + sr);
    E = kUtmFE + kUtmK0 * k.A * (etap + si);
}

// sinh and cosh from one expm1 (accurate near 0 as well)
RSAC_HD void dsinhcosh(double x, double &sh, double &ch) {
    const double em1 = expm1(x), e = 1.0 + em1;
    sh = 0.5 * (em1 + em1 / e);
    ch = 0.5 * (e + 1.0 / e);
}

// utm_inverse with the transcendental calls shared: one sincos + one expm1 per
// Clenshaw argument, sin/cos(2 chi) from sin chi.  Same series; differs from
// utm_inverse only by rounding (~1e-15 deg).  Used by the ray march.
RSAC_HD void utm_inverse_fast(const TmConst &k, const UtmZone &z, double E, double N, double &lon, double &lat) {
    const double kDeg = 57.29577951308232;
    const double xi = (N - z.fn) / (kUtmK0 * k.A);
    const double eta = (E - kUtmFE) / (kUtmK0 * k.A);
    double s2, c2, sh2, ch2;
    sincos(2.0 * xi, &s2, &c2);
    dsinhcosh(2.0 * eta, sh2, ch2);
    const double ar = 2.0 * c2 * ch2, ai = -2.0 * s2 * sh2;
    double y1r = 0.0, y1i = 0.0, y2r = 0.0, y2i = 0.0;
    for (int j = 5; j >= 0; --j) {
        const double yr = ar * y1r - ai * y1i - y2r + k.beta[j];
        const double yi = ar * y1i + ai * y1r - y2i;
        y2r = y1r; y2i = y1i;
        y1r = yr; y1i = yi;
    }
    const double br = s2 * ch2, bi = c2 * sh2;
    const double xip = xi - (y1r * br - y1i * bi), etap = eta - (y1r * bi + y1i * br);
    double sx, cx, she, che;
    sincos(xip, &sx, &cx);
    dsinhcosh(etap, she, che);
    const double sc = sx / che;                  // sin chi
    const double cc = dsqrt((1.0 - sc) * (1.0 + sc));  // cos chi >= 0
    const double chi = atan2(sc, cc);
    // delta series at chi: sum d_j sin(2 j chi), a = 2 cos(2 chi)
    const double a = 2.0 * (cc - sc) * (cc + sc);
    double y1 = 0.0, y2 = 0.0;
    for (int j = 5; j >= 0; --j) {
        const double y = a * y1 - y2 + k.delta[j];
        y2 = y1;
        y1 = y;
    }
    lat = (chi + y1 * (2.0 * sc * cc)) * kDeg;
    lon = (z.lon0 + atan2(she, cx)) * kDeg;
}

// The reference advances the ray by repeated addition, x_{s+1} = fl(x_s + c),
// c = fl(step * d) (main_v1.py:652-654).  Inside one binade, away from its
// ends, every such sum rounds onto the same grid u = ulp(x), so
// x_{s+j} = x_s + j * delta exactly, delta = fl(x_s + c) - x_s, unless the
// rounding of c onto the grid is a tie (then the even-rule alternates).
// stride_closed_form checks that for steps [0, W] from x and returns delta;
// false means the caller must add step by step.
RSAC_HD bool stride_closed_form(double x, double c, int W, double &delta) {
    if (x == 0.0 || !dfinite(x) || !dfinite(c)) return false;
    int ex;
    frexp(x, &ex);  // |x| in [2^(ex-1), 2^ex)
    const double lo = ldexp(1.0, ex - 1), hi = ldexp(1.0, ex), u = ldexp(1.0, ex - 53);
    const double ac = dabs(c);
    const double in_lo = lo + ac + 2.0 * u, in_hi = hi - ac - 2.0 * u;
    const double ax = dabs(x);
    if (!(ax >= in_lo && ax <= in_hi)) return false;
    const double d = (x + c) - x;      // exact: both in the binade
    if (dabs(c - d) == 0.5 * u) return false;  // tie: parity-dependent rounding
    const double end = x + (double)W * d;      // exact while inside the binade
    const double ae = dabs(end);
    if ((end < 0.0) != (x < 0.0) || !(ae >= in_lo && ae <= in_hi)) return false;
    delta = d;
    return true;
}

// A regular (lat, lon) grid as load_dem_data builds it (main_v1.py:430-433):
// lat_i = i * dy + y0, lon_j = j * dx + x0 (dy < 0 for north-up GDAL rasters).
struct DemGrid {
    const double *z;  // ny x nx, row-major (ReadAsArray)
    int ny, nx;
    double y0, dy, x0, dx;
};

// Linear interpolation at (lat, lon) as RegularGridInterpolator((dem_y, dem_x), z)
// evaluates it; false when the point is outside the grid (scipy raises, and
// ray_intersect_dem returns None, main_v1.py:644-647).
RSAC_HD bool dem_interp(const DemGrid &g, double lat, double lon, double &out) {
    const double ylo = g.dy > 0 ? g.y0 : (double)(g.ny - 1) * g.dy + g.y0;
    const double yhi = g.dy > 0 ? (double)(g.ny - 1) * g.dy + g.y0 : g.y0;
    const double xlo = g.dx > 0 ? g.x0 : (double)(g.nx - 1) * g.dx + g.x0;
    const double xhi = g.dx > 0 ? (double)(g.nx - 1) * g.dx + g.x0 : g.x0;
    if (!(lat >= ylo && lat <= yhi && lon >= xlo && lon <= xhi)) return false;
    double fy = (lat - g.y0) / g.dy, fx = (lon - g.x0) / g.dx;
    int i = (int)floor(fy), j = (int)floor(fx);
    i = i < 0 ? 0 : (i > g.ny - 2 ? g.ny - 2 : i);
    j = j < 0 ? 0 : (j > g.nx - 2 ? g.nx - 2 : j);
    const double yi = (double)i * g.dy + g.y0, yi1 = (double)(i + 1) * g.dy + g.y0;
    const double xj = (double)j * g.dx + g.x0, xj1 = (double)(j + 1) * g.dx + g.x0;
    const double ty = (lat - yi) / (yi1 - yi), tx = (lon - xj) / (xj1 - xj);
    const double *r0 = g.z + (int64_t)i * g.nx, *r1 = r0 + g.nx;
    out = (1.0 - ty) * ((1.0 - tx) * r0[j] + tx * r0[j + 1]) + ty * ((1.0 - tx) * r1[j] + tx * r1[j + 1]);
    return true;
}

// ray_intersect_dem (main_v1.py:635-656): march from `o` along `d` in steps of
// `step` m, at most n_steps times; hit = the first position, from step index
// min_steps on, whose height is at or below the DEM.  Returns 0 hit (pos set),
// 1 no hit within the search distance, 2 left the DEM (scipy bounds error).
RSAC_HD int dem_march(const TmConst &k, const UtmZone &z, const DemGrid &g, const double *o, const double *d,
                      int n_steps, double step, int min_steps, double *pos) {
    double p0 = o[0], p1 = o[1], p2 = o[2];
    for (int s = 0; s < n_steps; ++s) {
        double lon, lat, elev;
        utm_inverse(k, z, p0, p1, lon, lat);
        if (!dem_interp(g, lat, lon, elev)) return 2;
        if (s >= min_steps && p2 <= elev) {
            pos[0] = p0; pos[1] = p1; pos[2] = p2;
            return 0;
        }
        p0 = p0 + step * d[0];
        p1 = p1 + step * d[1];
        p2 = p2 + step * d[2];
    }
    return 1;
}

}  // namespace rsac
