"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's pixel -> ground-point march.

Only tests/ (and smoke()/bench's cpu_baseline) may import this module, as the checker.
The product (rsac.dem, kernel k_dem_march in csrc/rsac_geo.h) never does.

Follows main_v1.py:
  * :36-57   GeoCoordTransformer -- pyproj EPSG:4326 <-> EPSG:32650 (always_xy);
  * :425-465 load_dem_data -- RegularGridInterpolator((dem_y, dem_x), dem_array);
  * :547-573 pixel_to_ray;
  * :635-656 ray_intersect_dem -- restated loop by loop below.

pyproj is not installed in this image and the reference's repository holds no projected
coordinates (no UTM value is logged or stored), so the projection is PARITY UNPINNED against
pyproj.  It is restated independently of the kernel's formulation: direct (not Clenshaw) sums of
Krueger's series (Karney 2011, eqs. 35-36) and, for the inverse, Newton's iteration on the
conformal latitude (Karney 2011, eqs. 19-21) instead of the kernel's delta series.  The tests pin
it to a third, formula-free derivation: the meridian arc by quadrature on the central meridian,
(lon0, 0) -> (500000, 0), and conformality.  The interpolator is scipy's own
RegularGridInterpolator, as in the reference.
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import RegularGridInterpolator

A_WGS = 6378137.0
F_WGS = 1.0 / 298.257223563
K0 = 0.9996
FE = 500000.0


def _series():
    n = F_WGS / (2.0 - F_WGS)
    n2, n3, n4, n5, n6 = n ** 2, n ** 3, n ** 4, n ** 5, n ** 6
    A = A_WGS / (1 + n) * (1 + n2 / 4 + n4 / 64 + n6 / 256)
    alpha = [n / 2 - 2 * n2 / 3 + 5 * n3 / 16 + 41 * n4 / 180 - 127 * n5 / 288 + 7891 * n6 / 37800,
             13 * n2 / 48 - 3 * n3 / 5 + 557 * n4 / 1440 + 281 * n5 / 630 - 1983433 * n6 / 1935360,
             61 * n3 / 240 - 103 * n4 / 140 + 15061 * n5 / 26880 + 167603 * n6 / 181440,
             49561 * n4 / 161280 - 179 * n5 / 168 + 6601661 * n6 / 7257600,
             34729 * n5 / 80640 - 3418889 * n6 / 1995840,
             212378941 * n6 / 319334400]
    beta = [n / 2 - 2 * n2 / 3 + 37 * n3 / 96 - n4 / 360 - 81 * n5 / 512 + 96199 * n6 / 604800,
            n2 / 48 + n3 / 15 - 437 * n4 / 1440 + 46 * n5 / 105 - 1118711 * n6 / 3870720,
            17 * n3 / 480 - 37 * n4 / 840 - 209 * n5 / 4480 + 5569 * n6 / 90720,
            4397 * n4 / 161280 - 11 * n5 / 504 - 830251 * n6 / 7257600,
            4583 * n5 / 161280 - 108847 * n6 / 3991680,
            20648693 * n6 / 638668800]
    return A, np.array(alpha), np.array(beta)


_A, _ALPHA, _BETA = _series()
_E = np.sqrt(F_WGS * (2 - F_WGS))


def _lon0(zone):
    return np.radians(-183.0 + 6.0 * zone)


def wgs84_to_utm(lon, lat, zone=50, south=False):
    """Forward projection (EPSG:326zz/327zz), direct sums: Karney 2011 eqs. 7-9, 35."""
    phi = np.radians(np.asarray(lat, np.float64))
    dl = np.radians(np.asarray(lon, np.float64)) - _lon0(zone)
    tau = np.tan(phi)
    sig = np.sinh(_E * np.arctanh(_E * tau / np.sqrt(1 + tau ** 2)))
    taup = tau * np.sqrt(1 + sig ** 2) - sig * np.sqrt(1 + tau ** 2)
    xip = np.arctan2(taup, np.cos(dl))
    etap = np.arcsinh(np.sin(dl) / np.hypot(taup, np.cos(dl)))
    xi, eta = xip.copy(), etap.copy()
    for j in range(1, 7):
        xi = xi + _ALPHA[j - 1] * np.sin(2 * j * xip) * np.cosh(2 * j * etap)
        eta = eta + _ALPHA[j - 1] * np.cos(2 * j * xip) * np.sinh(2 * j * etap)
    return FE + K0 * _A * eta, (1e7 if south else 0.0) + K0 * _A * xi


def _tau_from_taup(taup):
    """Newton on tau'(tau) = taup (Karney 2011 eqs. 19-21)."""
    e2 = _E ** 2
    tau = taup / (1 - e2)
    for _ in range(8):
        sig = np.sinh(_E * np.arctanh(_E * tau / np.sqrt(1 + tau ** 2)))
        tp = tau * np.sqrt(1 + sig ** 2) - sig * np.sqrt(1 + tau ** 2)
        d = (1 - e2) * np.sqrt(1 + tp ** 2) * np.sqrt(1 + tau ** 2) / (1 + (1 - e2) * tau ** 2)
        tau = tau + (taup - tp) / d
    return tau


def utm_to_wgs84(easting, northing, zone=50, south=False):
    """Inverse projection, direct sums of the beta series: Karney 2011 eq. 36, then eq. 19-21."""
    xi = (np.asarray(northing, np.float64) - (1e7 if south else 0.0)) / (K0 * _A)
    eta = (np.asarray(easting, np.float64) - FE) / (K0 * _A)
    xip, etap = xi.copy(), eta.copy()
    for j in range(1, 7):
        xip = xip - _BETA[j - 1] * np.sin(2 * j * xi) * np.cosh(2 * j * eta)
        etap = etap - _BETA[j - 1] * np.cos(2 * j * xi) * np.sinh(2 * j * eta)
    taup = np.sin(xip) / np.hypot(np.sinh(etap), np.cos(xip))
    lat = np.degrees(np.arctan(_tau_from_taup(taup)))
    lon = np.degrees(_lon0(zone) + np.arctan2(np.sinh(etap), np.cos(xip)))
    return lon, lat


def meridian_northing(lat):
    """k0 x meridian arc by quadrature (formula-free pin for the central meridian)."""
    from scipy.integrate import quad
    e2 = _E ** 2
    m, _ = quad(lambda p: (1 - e2 * np.sin(p) ** 2) ** -1.5, 0.0, np.radians(lat), epsabs=0, epsrel=1e-13, limit=200)
    return K0 * A_WGS * (1 - e2) * m


def make_interpolator(z, y0, dy, x0, dx):
    """load_dem_data's interpolator (main_v1.py:431-433, 455)."""
    z = np.asarray(z, np.float64)
    dem_x = np.arange(z.shape[1]) * dx + x0
    dem_y = np.arange(z.shape[0]) * dy + y0
    return RegularGridInterpolator((dem_y, dem_x), z)


def ray_intersect_dem(ray_origin, ray_direction, interp, max_search_dist=10000, step=1, min_steps=150, zone=50,
                      south=False):
    """main_v1.py:635-656, one ray.  Returns (hit (3,) or None, status 0 hit / 1 none / 2 off the DEM)."""
    current_pos = np.array(ray_origin, dtype=np.float64)
    step_count = 0
    for _ in range(int(max_search_dist / step)):
        lon, lat = utm_to_wgs84(current_pos[0], current_pos[1], zone, south)
        try:
            dem_elev = interp((lat, lon))
        except ValueError:
            return None, 2
        if step_count >= min_steps and current_pos[2] <= dem_elev:
            return np.array([current_pos[0], current_pos[1], current_pos[2]]), 0
        current_pos[0] += step * ray_direction[0]
        current_pos[1] += step * ray_direction[1]
        current_pos[2] += step * ray_direction[2]
        step_count += 1
    return None, 1


def pixel_to_ray(pixel_x, pixel_y, K, R):
    """main_v1.py:547-573 (direction only)."""
    camera_ray = np.linalg.inv(K) @ np.array([pixel_x, pixel_y, 1.0])
    camera_ray /= np.linalg.norm(camera_ray)
    utm_ray = R.T @ camera_ray
    return utm_ray / np.linalg.norm(utm_ray)


def ray_intersect_dem_many(origins, directions, z, y0, dy, x0, dx, max_search_dist=10000, step=1, min_steps=150,
                           zone=50, south=False):
    """The same loop as ray_intersect_dem, advanced for all rays at once (numpy over rays, the
    per-ray arithmetic unchanged: the same projection, scipy's interpolation, the same += steps).
    Returns (hits (N,3) with NaN where none, status (N,) int8)."""
    z = np.asarray(z, np.float64)
    dem_x = np.arange(z.shape[1]) * dx + x0
    dem_y = np.arange(z.shape[0]) * dy + y0
    interp = RegularGridInterpolator((dem_y, dem_x), z, bounds_error=False, fill_value=np.nan)
    pos = np.array(origins, np.float64).reshape(-1, 3).copy()
    d = np.asarray(directions, np.float64).reshape(-1, 3)
    if pos.shape[0] == 1:
        pos = np.repeat(pos, d.shape[0], axis=0)
    n = d.shape[0]
    hits = np.full((n, 3), np.nan)
    status = np.ones(n, np.int8)
    live = np.arange(n)
    for s in range(int(max_search_dist / step)):
        if live.size == 0:
            break
        lon, lat = utm_to_wgs84(pos[live, 0], pos[live, 1], zone, south)
        elev = interp(np.c_[lat, lon])
        off = np.isnan(elev)
        status[live[off]] = 2
        hit = ~off & (s >= min_steps) & (pos[live, 2] <= elev)
        hits[live[hit]] = pos[live[hit]]
        status[live[hit]] = 0
        live = live[~off & ~hit]
        pos[live, 0] += step * d[live, 0]
        pos[live, 1] += step * d[live, 1]
        pos[live, 2] += step * d[live, 2]
    return hits, status
