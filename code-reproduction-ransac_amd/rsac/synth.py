"""Synthetic correspondence sets shaped like the reference's scene.

The reference georeferences a 2142x1620 photograph against UTM-50N points
(main_v1.py:889-890 builds ``pos3d``/``pixels``; testpro-K.py:198-225 hard-codes
12 of them).  No dataset ships beyond those 12 points, so benchmarks and the
large parity cases use seeded synthetic sets of the same geometry:

* intrinsics of main_v1.py:870-883 (f = 240 mm on a 127 x 178 mm plate,
  cx = 982.666819, cy = 697.950868, image 2142 x 1620);
* world points offset to UTM-like magnitudes (~7.39e5 E, ~2.888e6 N, ~700 m),
  so the float32 rounding that cv2.solvePnPRansac applies matters as it does
  in the reference;
* inliers = exact projection + N(0, sigma) px; outliers uniform in the image.
"""
from __future__ import annotations

import numpy as np

IMAGE_W, IMAGE_H = 2142, 1620
UTM_ORIGIN = np.array([739000.0, 2888500.0, 700.0])


def main_v1_K(width: int = IMAGE_W, height: int = IMAGE_H) -> np.ndarray:
    """K of main_v1.py:870-883."""
    fx = 240.0 / 127.0 * width
    fy = 240.0 / 178.0 * height
    return np.array([[fx, 0.0, 9.82666819e02], [0.0, fy, 6.97950868e02], [0.0, 0.0, 1.0]])


def random_rotation(rng: np.random.Generator) -> np.ndarray:
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(0.0, np.pi)
    kx = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * kx + (1 - np.cos(ang)) * (kx @ kx)


def pnp_problem(n: int, outlier_ratio: float = 0.5, seed: int = 0, noise_px: float = 1.0, K=None,
                depth=(300.0, 1500.0)):
    """One synthetic PnP problem.

    Returns dict(points3d (n,3) f64, points2d (n,2) f64, K, R, t, inlier (n,) bool).
    The ground-truth camera sits 500-1500 m from the cloud like the UTM scene.
    """
    rng = np.random.default_rng(seed)
    K = main_v1_K() if K is None else np.asarray(K, np.float64)
    R = random_rotation(rng)
    centre = UTM_ORIGIN + rng.uniform(-500.0, 500.0, size=3) * np.array([1.0, 1.0, 0.1])
    t = -R @ centre
    u = rng.uniform(0.0, IMAGE_W, size=n)
    v = rng.uniform(0.0, IMAGE_H, size=n)
    d = rng.uniform(depth[0], depth[1], size=n)
    Kinv = np.linalg.inv(K)
    rays = (Kinv @ np.stack([u, v, np.ones(n)])).T
    pc = rays * (d / rays[:, 2])[:, None]
    pw = (pc - t) @ R  # R^T (pc - t)
    proj = (K @ pc.T).T
    px = proj[:, :2] / proj[:, 2:3] + rng.normal(0.0, noise_px, size=(n, 2))
    n_out = int(round(outlier_ratio * n))
    out_idx = rng.permutation(n)[:n_out]
    inlier = np.ones(n, bool)
    inlier[out_idx] = False
    px[out_idx, 0] = rng.uniform(0.0, IMAGE_W, size=n_out)
    px[out_idx, 1] = rng.uniform(0.0, IMAGE_H, size=n_out)
    return dict(points3d=pw, points2d=px, K=K, R=R, t=t, inlier=inlier)


def homography_problem(n: int, outlier_ratio: float = 0.3, seed: int = 0, noise_px: float = 1.0):
    """Synthetic plane-to-image correspondences (src like the pos2 of main_v1.py:306-311)."""
    rng = np.random.default_rng(seed)
    src = rng.uniform(-1.0, 1.0, size=(n, 2)) * np.array([0.6, 0.2])
    H = np.array([[1500.0, 40.0, 1000.0], [30.0, -1400.0, 700.0], [0.05, 0.3, 1.0]])
    H = H + rng.normal(0.0, 1.0, size=(3, 3)) * np.array([[50, 20, 50], [20, 50, 50], [0.01, 0.02, 0]])
    hs = np.c_[src, np.ones(n)] @ H.T
    dst = hs[:, :2] / hs[:, 2:3] + rng.normal(0.0, noise_px, size=(n, 2))
    n_out = int(round(outlier_ratio * n))
    out_idx = rng.permutation(n)[:n_out]
    inlier = np.ones(n, bool)
    inlier[out_idx] = False
    dst[out_idx, 0] = rng.uniform(0.0, IMAGE_W, size=n_out)
    dst[out_idx, 1] = rng.uniform(0.0, IMAGE_H, size=n_out)
    return dict(src=src, dst=dst, H=H / H[2, 2], inlier=inlier)


# the 12 hard-coded correspondences and the known camera origin of testpro-K.py:198-234
TESTPRO_K_POS3D = np.array([
    [739031.2, 2888840.39, 726.0], [738995.929, 2888848.16, 724.0], [738963.052, 2888845.45, 721.0],
    [739173.616, 2888834.91, 697.0], [739077.689, 2888935.68, 726.0], [739033.253, 2888924.78, 726.0],
    [738973.016, 2888907.82, 723.0], [739136.184, 2889025.65, 705.0], [739179.948, 2888631.85, 702.0],
    [739140.769, 2888574.49, 702.0], [739312.871, 2888549.50, 720.0], [739249.159, 2888541.79, 707.0]])
TESTPRO_K_PIXELS = np.array([
    [582, 296], [402, 301], [272, 314], [1440, 467], [965, 296], [666, 265], [392, 283], [1583, 319],
    [729, 606], [169, 696], [1804, 672], [885, 824]], dtype=np.float64)
TESTPRO_K_FOCALS = [90, 100, 120, 150, 180, 210, 240, 300, 360]
TESTPRO_K_SENSORS = [(102, 127), (127, 178), (203, 254)]
TESTPRO_K_IMAGE = (2142, 1620)
TESTPRO_K_ORIGIN = np.array([739424.6, 2888281.18, 770.0])


def testpro_k_candidates():
    """The 27 intrinsics of the K sweep (testpro-K.py:58-70), in loop order."""
    out = []
    for f in TESTPRO_K_FOCALS:
        for (sw, sh) in TESTPRO_K_SENSORS:
            fx = f / (sw / TESTPRO_K_IMAGE[0])
            fy = f / (sh / TESTPRO_K_IMAGE[1])
            out.append(np.array([[fx, 0, TESTPRO_K_IMAGE[0] / 2], [0, fy, TESTPRO_K_IMAGE[1] / 2], [0, 0, 1.0]]))
    return out


def location_problem(n_features: int = 13, n_locations: int = 458, n_outliers: int = 2, n_unnoted: int = 1,
                     seed: int = 0, noise_px: float = 2.0, spacing: float = 150.0):
    """Camera-location search scene shaped like main_v1.py's (12 noted features, 458 candidate
    locations, main_v1.py:274, 862).

    Features lie 2-9 km ahead (first coordinate) of the true camera position.  From that position
    the direction ratios pos2 = (dz/dx, dy/dx) of main_v1.py:305-308 map to pixels by a homography
    (a rotating camera), plus noise; ``n_outliers`` pixels are random, ``n_unnoted`` are (0, 0).
    Candidates are a grid of ``spacing`` m around the true position, which is one of them."""
    rng = np.random.default_rng(seed)
    T = np.array([2888281.18, 739424.6, 770.0])
    pos3d = T + np.c_[rng.uniform(2000, 9000, n_features), rng.uniform(-4000, 4000, n_features),
                      rng.uniform(-200, 600, n_features)]
    d = pos3d - T
    ray = np.c_[d[:, 2] / d[:, 0], d[:, 1] / d[:, 0]]
    H = np.array([[0.0, 600.0, 1071.0], [-2500.0, 0.0, 900.0], [0.05, 0.02, 1.0]])
    H = H + rng.normal(size=(3, 3)) * np.array([[20, 20, 20], [20, 20, 20], [0.01, 0.01, 0]])
    hs = np.c_[ray, np.ones(n_features)] @ H.T
    pixels = hs[:, :2] / hs[:, 2:3] + rng.normal(0, noise_px, (n_features, 2))
    perm = rng.permutation(n_features)
    pixels[perm[:n_outliers]] = rng.uniform([0, 0], [IMAGE_W, IMAGE_H], (n_outliers, 2))
    pixels[perm[n_outliers:n_outliers + n_unnoted]] = 0.0
    side = int(np.ceil(np.sqrt(n_locations)))
    gi, gj = np.meshgrid(np.arange(side) - side // 2, np.arange(side) - side // 2, indexing="ij")
    grid = np.c_[gi.ravel(), gj.ravel()][:n_locations] * spacing
    locations = np.c_[T[0] + grid[:, 0], T[1] + grid[:, 1], T[2] + 30.0 * np.sin(grid[:, 0] / 700.0)]
    true_index = int(np.flatnonzero((grid[:, 0] == 0) & (grid[:, 1] == 0))[0])
    locations[true_index] = T
    return dict(pos3d=pos3d, pixels=pixels, locations=locations, true_index=true_index, H=H / H[2, 2])


def fundamental_problem(n: int = 50_000, outlier_ratio: float = 0.8, seed: int = 2, noise_px: float = 0.5):
    """Two synthetic views of a 3D scene (BASELINE.json configs[3]: 50k matches, 80 % outliers, seed 2).

    Returns dict(pts1, pts2 (N,2) pixels, F (3,3) ground truth, x2^T F x1 = 0, unit norm, inlier (N,) bool)."""
    rng = np.random.default_rng(seed)
    K = np.array([[1200.0, 0, 960.0], [0, 1200.0, 540.0], [0, 0, 1]])
    X = np.c_[rng.uniform(-30, 30, n), rng.uniform(-20, 20, n), rng.uniform(40, 120, n)]
    R2 = random_rotation(rng)
    # keep the second view close to the first: a small rotation
    w = rng.normal(size=3) * 0.08
    th = np.linalg.norm(w)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R2 = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    t2 = np.array([4.0, 0.5, 0.3]) + rng.normal(size=3) * 0.2
    x1 = X @ K.T
    x1 = x1[:, :2] / x1[:, 2:3]
    X2 = X @ R2.T + t2
    x2 = X2 @ K.T
    x2 = x2[:, :2] / x2[:, 2:3]
    x1 = x1 + rng.normal(0, noise_px, x1.shape)
    x2 = x2 + rng.normal(0, noise_px, x2.shape)
    n_out = int(round(outlier_ratio * n))
    out = rng.permutation(n)[:n_out]
    inlier = np.ones(n, bool)
    inlier[out] = False
    x2[out] = rng.uniform([0, 0], [1920, 1080], (n_out, 2))
    tx = np.array([[0, -t2[2], t2[1]], [t2[2], 0, -t2[0]], [-t2[1], t2[0], 0]])
    Ki = np.linalg.inv(K)
    F = Ki.T @ tx @ R2 @ Ki
    F = F / np.linalg.norm(F)
    return dict(pts1=x1, pts2=x2, F=F, inlier=inlier)



KULIANG_LONLAT = (119.3906, 26.0936)   # potential_camera_locations.csv area, UTM zone 50N


def camera_rotation(azimuth_deg: float, tilt_deg: float) -> np.ndarray:
    """R (UTM -> camera, x right, y down, z forward) of a camera looking at the azimuth (from
    north, clockwise) and tilted down by tilt_deg, as pixel_to_ray uses it (main_v1.py:569)."""
    az, tl = np.radians(azimuth_deg), np.radians(tilt_deg)
    z = np.array([np.sin(az) * np.cos(tl), np.cos(az) * np.cos(tl), -np.sin(tl)])
    x = np.array([np.cos(az), -np.sin(az), 0.0])
    y = np.cross(z, x)
    return np.stack([x, y, z])


def dem_problem(n_rays: int = 4096, seed: int = 0, half_extent_deg: float = 0.08, cell_deg: float = 1.0 / 3600,
                n_hills: int = 14, azimuth_deg: float = 40.0, tilt_deg: float = 0.0, height_above: float = 300.0):
    """A DEM scene for the ray march (main_v1.py:635-684; the reference's dem_data.tif is not shipped).

    DEM: north-up grid (GDAL geotransform gt = (x0, dx, 0, y0, 0, dy), dy < 0) of
    ``cell_deg`` cells (SRTM 1" by default) spanning +-half_extent_deg around Kuliang, smooth
    hills of 100-600 m over a 300 m plain.  Camera: at the centre, ``height_above`` m above the
    terrain, pose from ``camera_rotation``; rays = pixels uniform over the image, so a share of
    them points above the horizon (no hit, or off the DEM).

    Returns dict(z (ny,nx) f64, gt (6,), K, R, pixels (n,2), dirs (n,3), origin_lonlat (2,),
    origin_height); the caller projects origin_lonlat to UTM (rsac.dem.wgs84_to_utm)."""
    from .dem import pixel_to_ray
    rng = np.random.default_rng(seed)
    lon0, lat0 = KULIANG_LONLAT
    n = int(round(2 * half_extent_deg / cell_deg)) + 1
    gt = (lon0 - half_extent_deg, cell_deg, 0.0, lat0 + half_extent_deg, 0.0, -cell_deg)
    lat = np.arange(n) * gt[5] + gt[3]
    lon = np.arange(n) * gt[1] + gt[0]
    LA, LO = np.meshgrid(lat, lon, indexing="ij")
    z = np.full((n, n), 300.0)
    for _ in range(n_hills):
        cy, cx = lat0 + rng.uniform(-1, 1) * half_extent_deg, lon0 + rng.uniform(-1, 1) * half_extent_deg
        s = rng.uniform(0.004, 0.02)
        z += rng.uniform(100, 600) * np.exp(-((LA - cy) ** 2 + (LO - cx) ** 2) / (2 * s * s))
    K = main_v1_K()
    R = camera_rotation(azimuth_deg, tilt_deg)
    pixels = rng.uniform([0, 0], [IMAGE_W, IMAGE_H], (n_rays, 2))
    dirs = pixel_to_ray(pixels, K, R)
    return dict(z=z, gt=np.array(gt), K=K, R=R, pixels=pixels, dirs=dirs, origin_lonlat=np.array([lon0, lat0]),
                origin_height=float(z[n // 2, n // 2]) + height_above)
