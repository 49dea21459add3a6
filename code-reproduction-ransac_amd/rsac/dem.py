"""Pixel -> ground point: the reference's DEM ray march on the GPU.

Reference: main_v1.py:36-57 (GeoCoordTransformer, pyproj EPSG:4326 <-> EPSG:32650),
:425-465 (load_dem_data: RegularGridInterpolator over (lat, lon)), :547-573 (pixel_to_ray),
:635-656 (ray_intersect_dem: 1 m steps, up to 10 000, hit from step 150 on), :661-683
(pixel_to_geo).  The march is one GPU lane per ray (kernel k_dem_march, rsac_geo.h); the UTM
projection is Krueger's series to 6th order (pyproj is not installed here).

    dem = DemGrid.from_geotransform(dem_array, gdal_dataset.GetGeoTransform())
    hits, status = ray_intersect_dem(origins, directions, dem)      # many rays in one call
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

STATUS_HIT, STATUS_NO_HIT, STATUS_OFF_DEM = 0, 1, 2


def _ctx(device):
    return L.context(0 if device is None else device)


def _convert(inverse: bool, xy, zone: int, south: bool, device=None) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(xy, np.float64).reshape(-1, 2))
    out = np.zeros_like(a)
    ctx = _ctx(device)
    with ctx.lock:
        L.check(L.lib().rsac_utm_convert(ctx.handle, 1 if inverse else 0, a.ctypes.data, a.shape[0], int(zone),
                                         1 if south else 0, 0, out.ctypes.data, None))
    return out


def utm_to_wgs84(en, zone: int = 50, south: bool = False, device=None) -> np.ndarray:
    """(N,2) easting, northing -> (N,2) lon, lat in degrees (EPSG:326zz -> EPSG:4326, always_xy)."""
    return _convert(True, en, zone, south, device)


def wgs84_to_utm(lonlat, zone: int = 50, south: bool = False, device=None) -> np.ndarray:
    """(N,2) lon, lat in degrees -> (N,2) easting, northing."""
    return _convert(False, lonlat, zone, south, device)


class GeoCoordTransformer:
    """Drop-in for the reference's class (main_v1.py:36-57; EPSG:32650 = UTM zone 50N)."""

    def __init__(self, zone: int = 50, south: bool = False):
        self.zone, self.south = zone, south

    def wgs84_to_utm(self, lon, lat):
        e, n = wgs84_to_utm([[lon, lat]], self.zone, self.south)[0]
        if not (np.isfinite(e) and np.isfinite(n)):
            raise ValueError("Invalid UTM coordinates")
        return float(e), float(n)

    def utm_to_wgs84(self, easting, northing):
        lon, lat = utm_to_wgs84([[easting, northing]], self.zone, self.south)[0]
        if not (np.isfinite(lon) and np.isfinite(lat)):
            raise ValueError("Invalid WGS84 coordinates")
        return float(lon), float(lat)


@dataclass
class DemGrid:
    """A DEM on a regular (lat, lon) grid: z[i, j] at lat = i * dy + y0, lon = j * dx + x0."""
    z: np.ndarray
    y0: float
    dy: float
    x0: float
    dx: float

    @classmethod
    def from_geotransform(cls, array, gt):
        """As load_dem_data builds its axes from a GDAL geotransform (main_v1.py:431-433)."""
        return cls(np.ascontiguousarray(np.asarray(array, np.float64)), float(gt[3]), float(gt[5]), float(gt[0]),
                   float(gt[1]))

    def axes(self):
        ny, nx = self.z.shape
        return np.arange(ny) * self.dy + self.y0, np.arange(nx) * self.dx + self.x0


def pixel_to_ray(pixels, K, R) -> np.ndarray:
    """Unit UTM ray directions of pixels (main_v1.py:547-573): R^T normalize(K^-1 [u, v, 1])."""
    p = np.c_[np.asarray(pixels, np.float64).reshape(-1, 2), np.ones(len(np.asarray(pixels).reshape(-1, 2)))]
    cam = p @ np.linalg.inv(np.asarray(K, np.float64)).T
    cam /= np.linalg.norm(cam, axis=1, keepdims=True)
    utm = cam @ np.asarray(R, np.float64)  # (R^T cam)^T = cam^T R
    return utm / np.linalg.norm(utm, axis=1, keepdims=True)


def _is_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and x.is_cuda


def ray_intersect_dem(origins, directions, dem: DemGrid, max_search_dist: float = 10000, step: float = 1,
                      min_steps: int = 150, zone: int = 50, south: bool = False, device=None):
    """Batched ray_intersect_dem (main_v1.py:635-656).

    origins (N,3) or (3,) UTM positions (easting, northing, height), directions (N,3).
    Returns (hits (N,3), NaN where no hit; status (N,) int8: 0 hit, 1 none within the distance,
    2 left the DEM).  The reference returns None for status 1 and 2.
    ``directions`` as a CUDA tensor keeps everything on that device (the DEM is uploaded once and
    cached on the DemGrid) and returns CUDA tensors; the call then runs on the current stream.
    """
    if _is_cuda(directions):
        return _ray_intersect_dem_device(origins, directions, dem, max_search_dist, step, min_steps, zone, south)
    d = np.ascontiguousarray(np.asarray(directions, np.float64).reshape(-1, 3))
    o = np.asarray(origins, np.float64).reshape(-1, 3)
    if o.shape[0] == 1 and d.shape[0] != 1:
        o = np.repeat(o, d.shape[0], axis=0)
    o = np.ascontiguousarray(o)
    if o.shape != d.shape:
        raise ValueError("one origin per direction (or a single origin) required")
    ny, nx = dem.z.shape
    z = np.ascontiguousarray(dem.z, np.float64)
    hits = np.zeros_like(d)
    status = np.zeros(d.shape[0], np.int8)
    ctx = _ctx(device)
    with ctx.lock:
        L.check(L.lib().rsac_dem_ray_intersect(ctx.handle, o.ctypes.data, d.ctypes.data, d.shape[0], z.ctypes.data,
                                               ny, nx, dem.y0, dem.dy, dem.x0, dem.dx, int(zone), 1 if south else 0,
                                               float(max_search_dist), float(step), int(min_steps), 0,
                                               hits.ctypes.data, status.ctypes.data, None))
    return hits, status


def _ray_intersect_dem_device(origins, directions, dem, max_search_dist, step, min_steps, zone, south):
    import torch
    dev = directions.device
    d = directions.reshape(-1, 3).to(torch.float64).contiguous()
    o = torch.as_tensor(origins, dtype=torch.float64, device=dev).reshape(-1, 3)
    if o.shape[0] == 1 and d.shape[0] != 1:
        o = o.expand(d.shape[0], 3)
    o = o.contiguous()
    if o.shape != d.shape:
        raise ValueError("one origin per direction (or a single origin) required")
    cache = dem.__dict__.setdefault("_device_z", {})
    z = cache.get(dev.index)
    if z is None:
        z = torch.as_tensor(np.ascontiguousarray(dem.z, np.float64), device=dev)
        cache[dev.index] = z
    hits = torch.empty((d.shape[0], 3), dtype=torch.float64, device=dev)
    status = torch.empty(d.shape[0], dtype=torch.int8, device=dev)
    ny, nx = dem.z.shape
    ctx = _ctx(dev.index)
    with ctx.lock:
        L.check(L.lib().rsac_dem_ray_intersect(ctx.handle, o.data_ptr(), d.data_ptr(), d.shape[0], z.data_ptr(), ny, nx,
                                               dem.y0, dem.dy, dem.x0, dem.dx, int(zone), 1 if south else 0,
                                               float(max_search_dist), float(step), int(min_steps), L.F_DEVICE_IN,
                                               hits.data_ptr(), status.data_ptr(),
                                               C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return hits, status


def pixel_to_geo(pixels, K, R, ray_origin, dem: DemGrid, z_factors=None, **kw):
    """Batched pixel_to_geo (main_v1.py:661-683): ray per pixel, the z component scaled by the
    pixel's weighted optimisation factor (z_factors, (N,), default 1), renormalised, marched.
    Returns (hits (N,3), status (N,))."""
    d = pixel_to_ray(pixels, K, R)
    if z_factors is not None:
        d = d.copy()
        d[:, 2] *= np.asarray(z_factors, np.float64).reshape(-1)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
    return ray_intersect_dem(ray_origin, d, dem, **kw)
