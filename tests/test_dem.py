"""Pixel -> ground point: UTM projection and the DEM ray march.

CPU part: the oracle (oracle/dem_oracle.py) pinned without pyproj -- pyproj is absent and the
reference stores no projected coordinate, so the projection is "parity unpinned" against pyproj
and pinned instead to the meridian arc by quadrature, the zone origin, conformality and round
trips; the literal ray_intersect_dem loop (main_v1.py:635-656) against the batched oracle.

GPU part (marker gpu): rsac.dem (kernel k_dem_march, csrc/rsac_geo.h) against the oracle on the
same inputs.  Bar: projections within 1e-9 deg / 1e-6 m (two f64 evaluations of the same
series); march status identical and the hit the same step, except where the ray's height is
within 1e-6 m of the interpolated DEM at the deciding step (a last-ulp decision), where one
step either way is accepted.
"""
import numpy as np
import pytest

import dem_oracle as D
from rsac import synth


def test_oracle_zone_origin():
    e, n = D.wgs84_to_utm(117.0, 0.0)
    assert e == 500000.0 and n == 0.0
    lon, lat = D.utm_to_wgs84(500000.0, 0.0)
    assert abs(lon - 117.0) < 1e-12 and abs(lat) < 1e-12
    e, n = D.wgs84_to_utm(117.0, -10.0, south=True)
    assert abs(e - 500000.0) < 1e-9 and abs(n - (1e7 - D.meridian_northing(10.0))) < 1e-6


@pytest.mark.parametrize("lat", [1.0, 10.0, 26.09, 40.0, 60.0, 80.0])
def test_oracle_central_meridian_arc(lat):
    e, n = D.wgs84_to_utm(117.0, lat)
    assert abs(e - 500000.0) < 1e-9
    assert abs(n - D.meridian_northing(lat)) < 1e-6  # quadrature, no series


def test_oracle_round_trip_and_conformal():
    rng = np.random.default_rng(0)
    lon = 117.0 + rng.uniform(-3.5, 3.5, 400)
    lat = rng.uniform(-80, 84, 400)
    south = lat < 0
    for s in (False, True):
        k = south == s
        e, n = D.wgs84_to_utm(lon[k], lat[k], south=s)
        l2, b2 = D.utm_to_wgs84(e, n, south=s)
        assert np.max(np.abs(l2 - lon[k])) < 1e-11 and np.max(np.abs(b2 - lat[k])) < 1e-11
    # conformal: the scale is the same along the meridian and the parallel
    lo, la, h = 119.39, 26.09, 1e-6
    e0, n0 = D.wgs84_to_utm(lo, la)
    e1, n1 = D.wgs84_to_utm(lo + h, la)
    e2, n2 = D.wgs84_to_utm(lo, la + h)
    a = 6378137.0
    f = 1 / 298.257223563
    e2s = f * (2 - f)
    phi = np.radians(la)
    w = np.sqrt(1 - e2s * np.sin(phi) ** 2)
    k_par = np.hypot(e1 - e0, n1 - n0) / (np.radians(h) * a * np.cos(phi) / w)
    k_mer = np.hypot(e2 - e0, n2 - n0) / (np.radians(h) * a * (1 - e2s) / w ** 3)
    assert abs(k_par - k_mer) < 1e-7
    # convergence: the images of the meridian and parallel are orthogonal
    assert abs((e1 - e0) * (e2 - e0) + (n1 - n0) * (n2 - n0)) / (np.hypot(e1 - e0, n1 - n0) * np.hypot(e2 - e0, n2 - n0)) < 1e-7


def _scene(n_rays=64, seed=1, **kw):
    pr = synth.dem_problem(n_rays, seed=seed, **kw)
    e, n = D.wgs84_to_utm(*pr["origin_lonlat"])
    pr["origin"] = np.array([e, n, pr["origin_height"]])
    return pr


def test_oracle_batched_equals_literal_loop():
    pr = _scene(24, seed=3)
    gt = pr["gt"]
    hits, st = D.ray_intersect_dem_many(pr["origin"], pr["dirs"], pr["z"], gt[3], gt[5], gt[0], gt[1])
    interp = D.make_interpolator(pr["z"], gt[3], gt[5], gt[0], gt[1])
    assert set(st.tolist()) >= {0, 2}
    for i in range(len(st)):
        h, s = D.ray_intersect_dem(pr["origin"], pr["dirs"][i], interp)
        assert s == st[i]
        if s == 0:
            np.testing.assert_array_equal(h, hits[i])


def test_oracle_min_steps_and_short_search():
    pr = _scene(16, seed=4, height_above=25.0)
    gt = pr["gt"]
    # a ray straight down: underground from the first step, but the reference only tests from step 150
    down = np.array([[0.0, 0.0, -1.0]])
    h, s = D.ray_intersect_dem_many(pr["origin"], down, pr["z"], gt[3], gt[5], gt[0], gt[1])
    assert s[0] == 0 and abs(h[0, 2] - (pr["origin"][2] - 150.0)) < 1e-9
    # search distance shorter than min_steps: never a hit
    h, s = D.ray_intersect_dem_many(pr["origin"], down, pr["z"], gt[3], gt[5], gt[0], gt[1], max_search_dist=100)
    assert s[0] == 1


def test_pixel_to_ray_matches_reference_form():
    from rsac.dem import pixel_to_ray
    pr = _scene(8)
    d = pixel_to_ray(pr["pixels"], pr["K"], pr["R"])
    for i in range(8):
        np.testing.assert_allclose(d[i], D.pixel_to_ray(*pr["pixels"][i], pr["K"], pr["R"]), rtol=0, atol=1e-15)


# ------------------------------------------------------------------ GPU

def _check_march(pr, hits, st, oh, ost, step=1.0):
    gt = pr["gt"]
    interp = D.make_interpolator(pr["z"], gt[3], gt[5], gt[0], gt[1])
    bad = np.flatnonzero((st != ost) | ((st == 0) & np.any(hits != oh, axis=1)))
    for i in bad:
        # accepted only as a last-ulp decision: the oracle's and the kernel's hits are one step apart
        # and the height at the earlier of the two is within 1e-6 m of the DEM
        assert st[i] == 0 and ost[i] == 0, (i, st[i], ost[i])
        a, b = (hits[i], oh[i]) if hits[i][2] > oh[i][2] else (oh[i], hits[i])
        assert np.linalg.norm(a - b) <= step * (1 + 1e-9), (i, hits[i], oh[i])
        lon, lat = D.utm_to_wgs84(a[0], a[1])
        assert abs(a[2] - interp((lat, lon))) < 1e-6
    assert len(bad) <= max(1, len(st) // 100)


@pytest.mark.gpu
def test_gpu_utm_matches_oracle():
    from rsac import dem
    rng = np.random.default_rng(5)
    lon = 117.0 + rng.uniform(-3.5, 3.5, 5000)
    lat = rng.uniform(0, 84, 5000)
    en = dem.wgs84_to_utm(np.c_[lon, lat])
    e, n = D.wgs84_to_utm(lon, lat)
    assert np.max(np.abs(en[:, 0] - e)) < 1e-6 and np.max(np.abs(en[:, 1] - n)) < 1e-6
    ll = dem.utm_to_wgs84(en)
    l2, b2 = D.utm_to_wgs84(en[:, 0], en[:, 1])
    assert np.max(np.abs(ll[:, 0] - l2)) < 1e-9 and np.max(np.abs(ll[:, 1] - b2)) < 1e-9
    assert np.max(np.abs(ll[:, 0] - lon)) < 1e-9 and np.max(np.abs(ll[:, 1] - lat)) < 1e-9
    # southern zone, another zone number
    ens = dem.wgs84_to_utm(np.c_[lon - 60.0, -lat], zone=40, south=True)
    e, n = D.wgs84_to_utm(lon - 60.0, -lat, zone=40, south=True)
    assert np.max(np.abs(ens[:, 0] - e)) < 1e-6 and np.max(np.abs(ens[:, 1] - n)) < 1e-6
    t = dem.GeoCoordTransformer()
    assert t.wgs84_to_utm(117.0, 0.0) == (500000.0, 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_rays,kw", [(1, 300, {}), (2, 257, dict(tilt_deg=3.0, height_above=120.0)),
                                            (3, 64, dict(half_extent_deg=0.03, azimuth_deg=200.0)),
                                            (4, 2048, dict(tilt_deg=1.0))])
def test_gpu_ray_march_matches_oracle(seed, n_rays, kw):
    from rsac import dem
    pr = _scene(n_rays, seed=seed, **kw)
    gt = pr["gt"]
    g = dem.DemGrid.from_geotransform(pr["z"], gt)
    o = dem.wgs84_to_utm(pr["origin_lonlat"][None])[0]
    np.testing.assert_allclose(o, pr["origin"][:2], rtol=0, atol=1e-6)
    origin = pr["origin"]
    hits, st = dem.ray_intersect_dem(origin, pr["dirs"], g)
    oh, ost = D.ray_intersect_dem_many(origin, pr["dirs"], pr["z"], gt[3], gt[5], gt[0], gt[1])
    _check_march(pr, hits, st, oh, ost)


@pytest.mark.gpu
def test_gpu_ray_march_edges():
    from rsac import dem
    pr = _scene(8, seed=6, height_above=25.0)
    gt = pr["gt"]
    g = dem.DemGrid.from_geotransform(pr["z"], gt)
    o = pr["origin"]
    # straight down: hit exactly at step 150; short search: none; origin off the DEM: status 2
    down = np.array([[0.0, 0.0, -1.0]])
    h, s = dem.ray_intersect_dem(o, down, g)
    assert s[0] == 0 and h[0, 2] == D.ray_intersect_dem_many(o, down, pr["z"], gt[3], gt[5], gt[0], gt[1])[0][0, 2]
    h, s = dem.ray_intersect_dem(o, down, g, max_search_dist=100)
    assert s[0] == dem.STATUS_NO_HIT
    h, s = dem.ray_intersect_dem(o + np.array([1e5, 0, 0]), down, g)
    assert s[0] == dem.STATUS_OFF_DEM
    # empty input, steps of 2 m, min_steps 0
    h, s = dem.ray_intersect_dem(o, np.zeros((0, 3)), g)
    assert h.shape == (0, 3) and s.shape == (0,)
    h2, s2 = dem.ray_intersect_dem(o, pr["dirs"], g, step=2.0, min_steps=0)
    oh, ost = D.ray_intersect_dem_many(o, pr["dirs"], pr["z"], gt[3], gt[5], gt[0], gt[1], step=2.0, min_steps=0)
    _check_march(pr, h2, s2, oh, ost, step=2.0)


@pytest.mark.gpu
def test_gpu_ray_march_device_inputs_and_pixel_to_geo():
    import torch
    from rsac import dem
    import rsac._lib as L
    pr = _scene(200, seed=7)
    gt = pr["gt"]
    g = dem.DemGrid.from_geotransform(pr["z"], gt)
    hits, st = dem.ray_intersect_dem(pr["origin"], pr["dirs"], g)
    # device tensors through the C-ABI with RSAC_F_DEVICE_IN
    dev = torch.device("cuda:0")
    o_t = torch.tensor(np.repeat(pr["origin"][None], 200, 0), dtype=torch.float64, device=dev)
    d_t = torch.tensor(pr["dirs"], dtype=torch.float64, device=dev)
    z_t = torch.tensor(pr["z"], dtype=torch.float64, device=dev)
    h_t = torch.zeros((200, 3), dtype=torch.float64, device=dev)
    s_t = torch.zeros(200, dtype=torch.int8, device=dev)
    ctx = L.context(0)
    with ctx.lock:
        L.check(L.lib().rsac_dem_ray_intersect(ctx.handle, o_t.data_ptr(), d_t.data_ptr(), 200, z_t.data_ptr(),
                                               g.z.shape[0], g.z.shape[1], g.y0, g.dy, g.x0, g.dx, 50, 0, 10000.0,
                                               1.0, 150, L.F_DEVICE_IN, h_t.data_ptr(), s_t.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(s_t.cpu().numpy(), st)
    np.testing.assert_array_equal(h_t.cpu().numpy()[st == 0], hits[st == 0])
    # pixel_to_geo with unit factors = pixel_to_ray + march
    h2, s2 = dem.pixel_to_geo(pr["pixels"], pr["K"], pr["R"], pr["origin"], g)
    np.testing.assert_array_equal(s2, st)
    np.testing.assert_array_equal(h2[st == 0], hits[st == 0])
