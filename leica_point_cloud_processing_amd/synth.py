"""Deterministic input generation for tests and benchmarks (not part of the hot path).

* glibc rand() reproduced bit-for-bit (TYPE_3 additive feedback, srand(1) default), so the
  reference unit-test fixture -- CADToPointCloud(cube.ply, 5000) followed by
  Utils::rotateCloud(source, target, 0, 0, 0.175) (/root/reference/test/test_gicp_alignment.cpp:32-47)
  -- is regenerated exactly as the reference's gtest process would build it.
* CADToPointCloud::uniformSampling / randPSurface / randomPointTriangle
  (/root/reference/src/CADToPointCloud.cpp:101-190): area-weighted triangle sampling.
* A procedurally built asymmetric "aero part"  and a scan simulator
  (independent resample + Gaussian noise + rigid perturbation [+ occlusion]) for the
  100k .. 20M point configurations of BASELINE.json.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import math
import os
import struct

import numpy as np

RAND_MAX = 2147483647
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.cosf.restype = ctypes.c_float
_libm.cosf.argtypes = [ctypes.c_float]
_libm.sinf.restype = ctypes.c_float
_libm.sinf.argtypes = [ctypes.c_float]
_libm.sqrtf.restype = ctypes.c_float
_libm.sqrtf.argtypes = [ctypes.c_float]

f32 = np.float32


# ---------------------------------------------------------------------------------------
# glibc rand()
# ---------------------------------------------------------------------------------------
class GlibcRand:
    """glibc random_r TYPE_3 (x**31 + x**3 + 1), identical to rand() after srand(seed)."""

    def __init__(self, seed: int = 1):
        if seed == 0:
            seed = 1
        r = [0] * 34
        r[0] = seed
        for i in range(1, 31):
            hi, lo = divmod(r[i - 1], 127773)
            word = 16807 * lo - 2836 * hi
            if word < 0:
                word += 2147483647
            r[i] = word
        for i in range(31, 34):
            r[i] = r[i - 31]
        self._r = r
        for _ in range(34, 344):
            self._next_raw()

    def _next_raw(self) -> int:
        r = self._r
        v = (r[-31] + r[-3]) & 0xFFFFFFFF
        r.append(v)
        if len(r) > 64:
            del r[:-34]
        return v

    def rand(self) -> int:
        return self._next_raw() >> 1


# ---------------------------------------------------------------------------------------
# meshes
# ---------------------------------------------------------------------------------------
def read_ply(path: str):
    """Minimal PLY reader (ascii / binary_little_endian; float vertices, list faces)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header") + len(b"end_header")
    end = data.index(b"\n", end) + 1
    header = data[:end].decode("ascii").splitlines()
    fmt = None
    elements = []
    for line in header:
        tok = line.split()
        if not tok:
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append([tok[1], int(tok[2]), []])
        elif tok[0] == "property":
            elements[-1][2].append(tok[1:])
    nv = next(e[1] for e in elements if e[0] == "vertex")
    nf = next((e[1] for e in elements if e[0] == "face"), 0)
    vprops = next(e[2] for e in elements if e[0] == "vertex")
    body = data[end:]
    if fmt == "ascii":
        rows = body.decode("ascii").split("\n")
        verts = np.array([[float(x) for x in rows[i].split()[:3]] for i in range(nv)], dtype=np.float32)
        faces = [[int(x) for x in rows[nv + i].split()[1:]] for i in range(nf)]
    elif fmt == "binary_little_endian":
        tmap = {"float": "f", "float32": "f", "double": "d", "uchar": "B", "uint8": "B", "int": "i",
                "int32": "i", "uint": "I", "uint32": "I", "short": "h", "ushort": "H", "char": "b"}
        vfmt = "<" + "".join(tmap[p[0]] for p in vprops)
        vsz = struct.calcsize(vfmt)
        verts = np.array([struct.unpack_from(vfmt, body, i * vsz)[:3] for i in range(nv)], dtype=np.float32)
        off = nv * vsz
        fprops = next(e[2] for e in elements if e[0] == "face")[0]
        cnt_fmt, idx_fmt = "<" + tmap[fprops[1]], "<" + tmap[fprops[2]]
        faces = []
        for _ in range(nf):
            (cnt,) = struct.unpack_from(cnt_fmt, body, off)
            off += struct.calcsize(cnt_fmt)
            isz = struct.calcsize(idx_fmt)
            faces.append(list(struct.unpack_from("<" + idx_fmt[1:] * cnt, body, off)))
            off += isz * cnt
    else:
        raise ValueError(f"unsupported PLY format {fmt}")
    return verts, triangulate(faces)


def read_obj(path: str):
    """Minimal OBJ reader (v / f records, 1-based indices, `v//vn` forms), like vtkOBJReader."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "v":
                verts.append([float(t) for t in tok[1:4]])
            elif tok[0] == "f":
                faces.append([int(t.split("/")[0]) - 1 for t in tok[1:]])
    return np.array(verts, dtype=np.float32), triangulate(faces)


def triangulate(faces):
    """vtkTriangleFilter for convex polygons: fan triangulation, triangles pass through."""
    tris = []
    for f in faces:
        for i in range(1, len(f) - 1):
            tris.append([f[0], f[i], f[i + 1]])
    return np.array(tris, dtype=np.int64).reshape(-1, 3)


def triangle_areas(verts: np.ndarray, tris: np.ndarray) -> np.ndarray:
    """vtkTriangle::TriangleArea in double: 0.25*sqrt(|4ac - (a-b+c)^2|), squared edge lengths."""
    v = verts.astype(np.float64)
    p1, p2, p3 = v[tris[:, 0]], v[tris[:, 1]], v[tris[:, 2]]
    a = ((p1 - p2) ** 2).sum(1)
    b = ((p2 - p3) ** 2).sum(1)
    c = ((p3 - p1) ** 2).sum(1)
    return 0.25 * np.sqrt(np.abs(4.0 * a * c - (a - b + c) * (a - b + c)))


def cad_sample_reference(verts: np.ndarray, tris: np.ndarray, n: int, rng: GlibcRand) -> np.ndarray:
    """CADToPointCloud::uniformSampling with glibc rand(), scalar float32 arithmetic (exact)."""
    cum = np.cumsum(triangle_areas(verts, tris))
    total = float(cum[-1])
    out = np.empty((n, 3), dtype=np.float32)
    inv = 1.0 / (RAND_MAX + 1.0)
    for i in range(n):
        r = f32(rng.rand() * inv * total)
        el = int(np.searchsorted(cum, float(r), side="left"))
        A, B, C = verts[tris[el, 0]], verts[tris[el, 1]], verts[tris[el, 2]]
        r1 = f32(rng.rand() * inv)
        r2 = f32(rng.rand() * inv)
        r1sqr = f32(_libm.sqrtf(float(r1)))
        one_min_r1 = f32(f32(1) - r1sqr)
        one_min_r2 = f32(f32(1) - r2)
        for d in range(3):
            a = f32(A[d] * one_min_r1)
            b = f32(B[d] * one_min_r2)
            out[i, d] = f32(f32(r1sqr * f32(f32(r2 * C[d]) + b)) + a)
    return out


def cad_sample_fast(verts: np.ndarray, tris: np.ndarray, n: int, seed: int, chunk: int = 1 << 22) -> np.ndarray:
    """Same sampling scheme, vectorised with numpy PCG64 (for the 1e5..2e7 point configs)."""
    cum = np.cumsum(triangle_areas(verts, tris))
    total = float(cum[-1])
    g = np.random.Generator(np.random.PCG64(seed))
    v = verts.astype(np.float32)
    out = np.empty((n, 3), dtype=np.float32)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        r = (g.random(m) * total).astype(np.float32)
        el = np.minimum(np.searchsorted(cum, r.astype(np.float64), side="left"), len(tris) - 1)
        r1 = g.random(m).astype(np.float32)
        r2 = g.random(m).astype(np.float32)
        r1s = np.sqrt(r1)
        a = v[tris[el, 0]] * (np.float32(1) - r1s)[:, None]
        b = v[tris[el, 1]] * (np.float32(1) - r2)[:, None]
        c = r1s[:, None] * (r2[:, None] * v[tris[el, 2]] + b) + a
        out[s:s + m] = c
    return out


# ---------------------------------------------------------------------------------------
# rigid transforms with Eigen float semantics
# ---------------------------------------------------------------------------------------
def _quat_axis(angle: float, axis: int):
    ha = f32(f32(0.5) * f32(angle))
    s = f32(_libm.sinf(float(ha)))
    q = [f32(_libm.cosf(float(ha))), f32(0), f32(0), f32(0)]
    q[1 + axis] = s
    return q


def _quat_mul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return [
        f32(f32(f32(f32(aw * bw) - f32(ax * bx)) - f32(ay * by)) - f32(az * bz)),
        f32(f32(f32(f32(aw * bx) + f32(ax * bw)) + f32(ay * bz)) - f32(az * by)),
        f32(f32(f32(f32(aw * by) + f32(ay * bw)) + f32(az * bx)) - f32(ax * bz)),
        f32(f32(f32(f32(aw * bz) + f32(az * bw)) + f32(ax * by)) - f32(ay * bx)),
    ]


def _quat_matrix(q) -> np.ndarray:
    w, x, y, z = q
    tx, ty, tz = f32(2 * x), f32(2 * y), f32(2 * z)
    twx, twy, twz = f32(tx * w), f32(ty * w), f32(tz * w)
    txx, txy, txz = f32(tx * x), f32(ty * x), f32(tz * x)
    tyy, tyz, tzz = f32(ty * y), f32(tz * y), f32(tz * z)
    R = np.array([
        [f32(1) - f32(tyy + tzz), f32(txy - twz), f32(txz + twy)],
        [f32(txy + twz), f32(1) - f32(txx + tzz), f32(tyz - twx)],
        [f32(txz - twy), f32(tyz + twx), f32(1) - f32(txx + tyy)],
    ], dtype=np.float32)
    return R


def rotate_cloud_matrix(roll: float, pitch: float, yaw: float) -> np.ndarray:
    """Utils::rotateCloud's T (/root/reference/src/Utils.cpp:215-232):
    q = AngleAxisf(roll,X) * AngleAxisf(pitch,Y) * AngleAxisf(yaw,Z); T = [q.matrix() 0; 0 1]."""
    q = _quat_mul(_quat_mul(_quat_axis(roll, 0), _quat_axis(pitch, 1)), _quat_axis(yaw, 2))
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = _quat_matrix(q)
    return T


def transform_points(T: np.ndarray, xyz: np.ndarray) -> np.ndarray:
    """pcl::transformPointCloud xyz: ((T00 x + T01 y) + T02 z) + T03 in float32, no FMA."""
    T = np.asarray(T, dtype=np.float32)
    xyz = np.asarray(xyz, dtype=np.float32)
    out = np.empty_like(xyz)
    for r in range(3):
        a = T[r, 0] * xyz[:, 0]
        a = a + T[r, 1] * xyz[:, 1]
        a = a + T[r, 2] * xyz[:, 2]
        out[:, r] = a + T[r, 3]
    return out


def axis_angle_matrix(axis, angle: float, center=(0.0, 0.0, 0.0), t=(0.0, 0.0, 0.0)) -> np.ndarray:
    """4x4 (float64) rotation about `axis` through `center`, then translation t."""
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) + math.sin(angle) * K + (1 - math.cos(angle)) * K @ K
    c = np.asarray(center, dtype=np.float64)
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = c - R @ c + np.asarray(t, dtype=np.float64)
    return T


# ---------------------------------------------------------------------------------------
# reference unit-test fixture (test_gicp_alignment.cpp)
# ---------------------------------------------------------------------------------------
def filter_test_cube(rng: "GlibcRand", dim: float = 5.0, nsamples: int = 5000, x: float = 0.0) -> np.ndarray:
    """TestFilter::cubePointCloud (/root/reference/test/test_filter.cpp:36-49): nsamples points
    x + dim * (double)rand() / (double)RAND_MAX per coordinate (double arithmetic, stored as float),
    drawing x, y, z in that order from the glibc rand() stream `rng`."""
    out = np.empty((nsamples, 3), np.float32)
    for i in range(nsamples):
        for d in range(3):
            out[i, d] = np.float32(x + dim * float(rng.rand()) / 2147483647.0)
    return out


def cube_fixture(ply_path: str, n: int = 5000, yaw: float = 0.175):
    """(source_xyz, target_xyz, T_rot): source = CADToPointCloud(cube.ply, n) with glibc rand()
    from its default seed, target = Utils::rotateCloud(source, 0, 0, yaw)."""
    verts, tris = read_ply(ply_path)
    src = cad_sample_reference(verts, tris, n, GlibcRand(1))
    T = rotate_cloud_matrix(0.0, 0.0, yaw)
    return src, transform_points(T, src), T


def cube_ply_vs_obj(ply_path: str, obj_path: str, n: int = 5000, yaw: float = 0.175):
    """BASELINE.json configs[0] ("test/cube.ply vs test/cube.obj-sampled"): source =
    CADToPointCloud(cube.ply, n) with glibc rand() from its default seed (as test_gicp_alignment.cpp:
    32-47), target = CADToPointCloud(cube.obj, n) drawn from the SAME generator afterwards (one
    process sampling both files, CADToPointCloud.cpp:35-62; vtkOBJReader -> vtkTriangleFilter),
    rotated by Utils::rotateCloud(0, 0, yaw).  Two independent samplings of the same cube: no point
    of the source has an exact partner in the target, unlike the ply-only fixture."""
    rng = GlibcRand(1)
    v, t = read_ply(ply_path)
    src = cad_sample_reference(v, t, n, rng)
    v2, t2 = read_obj(obj_path)
    tgt0 = cad_sample_reference(v2, t2, n, rng)
    T = rotate_cloud_matrix(0.0, 0.0, yaw)
    return src, transform_points(T, tgt0), T


# ---------------------------------------------------------------------------------------
# synthetic aero part
# ---------------------------------------------------------------------------------------
PART_CENTER = (1.7, 2.9, 2.8)  # launch/leica_point_cloud_processing.launch:12-14


def _box(lo, hi, step):
    """Closed axis-aligned box as triangles, each face subdivided to edges <= step."""
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    verts, tris = [], []

    def face(origin, u, v):
        nu = max(1, int(math.ceil(np.linalg.norm(u) / step)))
        nv = max(1, int(math.ceil(np.linalg.norm(v) / step)))
        base = len(verts)
        for j in range(nv + 1):
            for i in range(nu + 1):
                verts.append(origin + u * (i / nu) + v * (j / nv))
        for j in range(nv):
            for i in range(nu):
                a = base + j * (nu + 1) + i
                tris.append([a, a + 1, a + nu + 2])
                tris.append([a, a + nu + 2, a + nu + 1])

    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    face(lo, ey, ex)                      # bottom
    face(lo + ez, ex, ey)                 # top
    face(lo, ex, ez)                      # front
    face(lo + ey, ez, ex)                 # back
    face(lo, ez, ey)                      # left
    face(lo + ex, ey, ez)                 # right
    return np.array(verts), np.array(tris)


def _cylinder(cx, cy, z0, z1, radius, seg, step):
    verts, tris = [], []
    nz = max(1, int(math.ceil((z1 - z0) / step)))
    for k in range(nz + 1):
        z = z0 + (z1 - z0) * k / nz
        for s in range(seg):
            a = 2 * math.pi * s / seg
            verts.append([cx + radius * math.cos(a), cy + radius * math.sin(a), z])
    for k in range(nz):
        for s in range(seg):
            a, b = k * seg + s, k * seg + (s + 1) % seg
            tris.append([a, b, b + seg])
            tris.append([a, b + seg, a + seg])
    for z, flip in ((z0, True), (z1, False)):  # caps as fans
        c = len(verts)
        verts.append([cx, cy, z])
        ring0 = 0 if z == z0 else nz * seg
        for s in range(seg):
            a, b = ring0 + s, ring0 + (s + 1) % seg
            tris.append([c, b, a] if flip else [c, a, b])
    return np.array(verts), np.array(tris)


def aero_part_mesh(step: float = 0.1):
    """Asymmetric 4.1 m part: skin plate, three unevenly spaced frames, a stringer, a tilted
    flange and a cylindrical boss.  Centred at PART_CENTER; >= 2000 triangles."""
    parts = [
        _box((-2.05, -0.65, -0.02), (2.05, 0.65, 0.02), step),          # skin
        _box((-1.55, -0.65, 0.02), (-1.51, 0.65, 0.37), step),          # frame 1
        _box((-0.60, -0.65, 0.02), (-0.56, 0.65, 0.30), step),          # frame 2
        _box((0.90, -0.65, 0.02), (0.94, 0.65, 0.42), step),            # frame 3
        _box((-2.05, 0.33, 0.02), (2.05, 0.37, 0.22), step),            # stringer
        _cylinder(1.50, -0.30, 0.02, 0.52, 0.18, 48, step),             # boss
    ]
    # tilted flange at the left end: box rotated 30 deg about y
    fv, ft = _box((-0.25, -0.65, -0.015), (0.25, 0.65, 0.015), step)
    ang = math.radians(30.0)
    Ry = np.array([[math.cos(ang), 0, math.sin(ang)], [0, 1, 0], [-math.sin(ang), 0, math.cos(ang)]])
    fv = fv @ Ry.T + np.array([-2.25, 0.0, 0.12])
    parts.append((fv, ft))
    verts, tris, base = [], [], 0
    for v, t in parts:
        verts.append(v)
        tris.append(t + base)
        base += len(v)
    V = np.concatenate(verts) + np.asarray(PART_CENTER)
    return V.astype(np.float32), np.concatenate(tris).astype(np.int64)


def _unit_dirs(g: np.random.Generator, m: int) -> np.ndarray:
    v = g.normal(size=(m, 3))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def clutter_and_debris(verts, tris, n_clutter: int, n_debris: int, clusters: int, seed: int) -> np.ndarray:
    """Scan points with no CAD partner -- what FODDetectionState subtracts the CAD for
    (/root/reference/src/LeicaStateMachine.cpp:180-189):
      * clutter: surface points pushed 5-30 cm off the part along a random direction (fixtures,
        the floor, the scanner's mixed pixels), far beyond the 4 cm gate of GICPAlignment
        (/root/reference/src/GICPAlignment.cpp:31) unless another face of the part lies near;
      * debris: `clusters` blobs (uniform in balls of radius 0.5-2 cm) whose centres sit 0.5-5 cm
        off a surface point -- partly inside, partly outside the gate.
    Rows are in part coordinates (before noise and T_true), float64."""
    g = np.random.Generator(np.random.PCG64(seed))
    out = []
    if n_clutter > 0:
        base = cad_sample_fast(verts, tris, n_clutter, seed + 1).astype(np.float64)
        out.append(base + _unit_dirs(g, n_clutter) * g.uniform(0.05, 0.30, size=(n_clutter, 1)))
    if n_debris > 0:
        clusters = max(1, min(clusters, n_debris))
        ctr = cad_sample_fast(verts, tris, clusters, seed + 2).astype(np.float64)
        ctr += _unit_dirs(g, clusters) * g.uniform(0.005, 0.05, size=(clusters, 1))
        rad = g.uniform(0.005, 0.02, size=clusters)
        which = np.arange(n_debris) % clusters
        r = rad[which][:, None] * np.cbrt(g.uniform(size=(n_debris, 1)))
        out.append(ctr[which] + _unit_dirs(g, n_debris) * r)
    return np.concatenate(out) if out else np.zeros((0, 3))


def scan_vs_cad(n_scan: int, n_cad: int, noise: float = 5e-4, angle: float = 0.02,
                axis=(0.3, 0.5, 0.81), t=(0.010, -0.005, 0.008), occlusion: float = 0.0,
                seeds=(1, 2, 3), clutter: float = 0.0, debris: int = 0, debris_clusters: int = 40):
    """(scan_xyz, cad_xyz, T_true): CAD cloud = area-weighted sample (seed 1); scan =
    independent resample (seed 2) + N(0, noise^2) per axis (seed 3), moved by T_true (a
    rotation about `axis` through PART_CENTER plus t).  `occlusion` drops that fraction of
    the surface area (triangles with the largest x) from the scan.  `clutter` (a fraction of
    n_scan) and `debris` (points in `debris_clusters` blobs) replace that many surface samples
    by points without a CAD partner (clutter_and_debris, seed 4); they are spread through the
    scan's order like the surface points.  clutter = debris = 0 gives the same clouds as before."""
    verts, tris = aero_part_mesh()
    cad = cad_sample_fast(verts, tris, n_cad, seeds[0])
    stris = tris
    if occlusion > 0:
        cx = verts[tris].mean(axis=1)[:, 0]
        order = np.argsort(cx)
        area = triangle_areas(verts, tris)[order]
        keep = np.cumsum(area) <= (1.0 - occlusion) * area.sum()
        stris = tris[order[keep]]
    n_clutter = int(round(clutter * n_scan))
    n_extra = n_clutter + int(debris)
    if n_extra > n_scan:
        raise ValueError("clutter + debris exceed the scan size")
    scan = cad_sample_fast(verts, stris, n_scan - n_extra, seeds[1]).astype(np.float64)
    if n_extra:
        extra = clutter_and_debris(verts, stris, n_clutter, int(debris), debris_clusters, 4)
        pos = np.random.Generator(np.random.PCG64(5)).permutation(n_scan)[:n_extra]
        full = np.empty((n_scan, 3))
        mask = np.ones(n_scan, bool)
        mask[pos] = False
        full[mask] = scan
        full[pos] = extra
        scan = full
    g = np.random.Generator(np.random.PCG64(seeds[2]))
    for s in range(0, n_scan, 1 << 22):
        m = min(1 << 22, n_scan - s)
        scan[s:s + m] += g.normal(0.0, noise, size=(m, 3))
    T = axis_angle_matrix(axis, angle, PART_CENTER, t)
    scan = scan @ T[:3, :3].T + T[:3, 3]
    return scan.astype(np.float32), cad, T


def repo_root() -> str:
    return os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
