"""Dense pose verification (InLoc "DensePV") for NC-Net pose candidates.

The reference re-ranks the top-10 P3P poses of each query by how well a view
synthesised from the database scan at that pose matches the query image
(lib_matlab/ht_top10_NC4D_PV_localization.m, at_pv_wrapper.m,
parfor_nc4d_PV.m).  Per (query, cutout, pose):

1. query image downsampled by 1/8, intrinsics K = [f/8, 0, w/2; 0, f/8, h/2; 0, 0, 1]
   (parfor_nc4d_PV.m:2,11-13);
2. the scan point cloud (RGB + XYZ, moved by the scan's P_after transform,
   at_pv_wrapper.m:9-14) is z-buffer projected through K*P into an RGB and an
   XYZ image; pixels no point lands on are NaN (``ht_Points2Persp``, :14-15);
3. both grey images are normalised over the valid mask, the holes of the
   synthetic one in-painted first (:19-23);
4. dense SIFT at bin size 8 / step 4 (``vl_phow``), RootSIFT, and the score is
   1 / median of the descriptor distances at valid keypoints (:26-34);
5. the top-10 candidates are sorted by score, descending
   (ht_top10_NC4D_PV_localization.m:63-67).

``ht_Points2Persp``, ``image_normalization``, ``inpaint_nans`` and ``vl_phow``
come from InLoc_demo / VLFeat, which are not part of the reference; they are
re-implemented here in torch (CPU or GPU) from their documented behaviour:
nearest-point z-buffer splatting, zero-mean / unit-variance normalisation on
the valid mask, diffusion in-painting, and a VLFeat-style dense SIFT
(Gaussian pre-smoothing sigma = size / 6, 8 orientation bins with linear
orientation interpolation, bilinear 4x4 spatial binning, L2 -> clamp 0.2 ->
L2).  Scores are therefore "parity unpinned" against MATLAB; the re-ranking
logic and the I/O contract are the reference's.
"""
from __future__ import annotations

import math
import os
import re

import numpy as np
import torch
import torch.nn.functional as F

DS_LEVEL = 1.0 / 8.0


# ---------------------------------------------------------------------------
# rendering
def points_to_perspective(rgb: torch.Tensor, xyz: torch.Tensor, KP: torch.Tensor, h: int, w: int):
    """Z-buffered projection of a coloured point cloud (``ht_Points2Persp``).

    rgb [N, 3] (any range), xyz [N, 3] world points, KP [3, 4] = K @ [R | t].
    Returns (rgb_img [h, w, 3], xyz_img [h, w, 3]) with NaN where no point
    projects; each pixel keeps its nearest point in front of the camera.
    """
    dev = xyz.device
    Xh = torch.cat([xyz.double(), torch.ones(xyz.shape[0], 1, dtype=torch.float64, device=dev)], 1)
    p = Xh @ KP.double().T                       # [N, 3]
    z = p[:, 2]
    ok = z > 1e-9
    u = torch.floor(p[:, 0] / z.clamp_min(1e-12)).long()   # pixel (col) index, 0-based
    v = torch.floor(p[:, 1] / z.clamp_min(1e-12)).long()
    ok &= (u >= 0) & (u < w) & (v >= 0) & (v < h)
    idx = (v * w + u)[ok]
    zk = z[ok]
    src = torch.nonzero(ok).squeeze(1)
    zbuf = torch.full((h * w,), float("inf"), dtype=torch.float64, device=dev)
    zbuf.scatter_reduce_(0, idx, zk, reduce="amin")
    win = zk <= zbuf[idx]                        # this point is the nearest one of its pixel
    pix, pts = idx[win], src[win]
    rgb_img = torch.full((h * w, 3), float("nan"), dtype=torch.float32, device=dev)
    xyz_img = torch.full((h * w, 3), float("nan"), dtype=torch.float32, device=dev)
    rgb_img[pix] = rgb[pts].float()
    xyz_img[pix] = xyz[pts].float()
    return rgb_img.view(h, w, 3), xyz_img.view(h, w, 3)


def rgb2gray(img: torch.Tensor) -> torch.Tensor:
    """MATLAB rgb2gray weights on an [h, w, 3] tensor."""
    return img[..., 0] * 0.2989 + img[..., 1] * 0.5870 + img[..., 2] * 0.1140


def inpaint_nans(img: torch.Tensor, iters: int = 50) -> torch.Tensor:
    """Fill NaN pixels (the role of ``inpaint_nans``): grow the known region
    by 4-neighbour averaging until every pixel is set, then relax the filled
    pixels towards the average of their neighbours (a discrete Laplace
    in-painting with the known pixels as boundary values)."""
    known = ~torch.isnan(img)
    if bool(known.all()) or not bool(known.any()):
        return torch.nan_to_num(img, nan=0.0)
    k = torch.tensor([[0, 1, 0], [1, 0, 1], [0, 1, 0]], dtype=img.dtype, device=img.device)[None, None]
    nb = lambda t: F.conv2d(F.pad(t, (1, 1, 1, 1), mode="replicate"), k)   # noqa: E731
    m = known.to(img.dtype)[None, None]
    x = torch.where(known, img, torch.zeros_like(img))[None, None]
    filled = m.clone()
    while not bool((filled > 0).all()):
        s, c = nb(x * filled), nb(filled)
        grow = (filled == 0) & (c > 0)
        x = torch.where(grow, s / c.clamp_min(1e-12), x)
        filled = torch.where(grow, torch.ones_like(filled), filled)
    for _ in range(iters):
        x = torch.where(m > 0, x, nb(x) / 4.0)
    return x[0, 0]


def image_normalization(img: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Zero-mean, unit-variance over the valid mask (``image_normalization``),
    rescaled to [0, 1] for the descriptor."""
    vals = img[mask]
    if vals.numel() < 2:
        return torch.zeros_like(img)
    x = (img - vals.mean()) / vals.std().clamp_min(1e-6)
    lo, hi = x[mask].min(), x[mask].max()
    return ((x - lo) / (hi - lo).clamp_min(1e-6)).clamp(0, 1)


# ---------------------------------------------------------------------------
# dense SIFT
def dense_sift(img: torch.Tensor, size: int = 8, step: int = 4, magnif: float = 6.0, nori: int = 8):
    """VLFeat-style dense SIFT (``vl_phow(I, 'sizes', size, 'step', step)``).

    img [h, w] in [0, 1].  Returns (frames [2, n] = (x, y) 0-based keypoint
    centres, descriptors [128, n] in [0, 1]).  A descriptor is 4 x 4 spatial
    bins of ``size`` px x ``nori`` orientations; gradient magnitudes vote
    with linear orientation interpolation and bilinear spatial weights.
    """
    dev, dt = img.device, torch.float32
    x = img.to(dt)[None, None]
    sigma = size / magnif
    r = max(1, int(math.ceil(3 * sigma)))
    t = torch.arange(-r, r + 1, device=dev, dtype=dt)
    gk = torch.exp(-0.5 * (t / sigma) ** 2)
    gk = gk / gk.sum()
    x = F.conv2d(F.pad(x, (r, r, 0, 0), mode="replicate"), gk.view(1, 1, 1, -1))
    x = F.conv2d(F.pad(x, (0, 0, r, r), mode="replicate"), gk.view(1, 1, -1, 1))
    xp = F.pad(x, (1, 1, 1, 1), mode="replicate")
    gx = 0.5 * (xp[..., 1:-1, 2:] - xp[..., 1:-1, :-2])
    gy = 0.5 * (xp[..., 2:, 1:-1] - xp[..., :-2, 1:-1])
    mag = torch.sqrt(gx * gx + gy * gy)[0, 0]
    ang = torch.atan2(gy, gx)[0, 0] % (2 * math.pi)
    # linear interpolation between the two nearest orientation bins
    fb = ang / (2 * math.pi) * nori
    b0 = torch.floor(fb).long() % nori
    w1 = fb - torch.floor(fb)
    H, W = mag.shape
    omap = torch.zeros(nori, H, W, device=dev, dtype=dt)
    omap.scatter_add_(0, b0[None], (mag * (1 - w1))[None])
    omap.scatter_add_(0, ((b0 + 1) % nori)[None], (mag * w1)[None])
    # bilinear (triangular) spatial weighting of width 2*size per bin
    tri = 1 - (torch.arange(-size + 1, size, device=dev, dtype=dt).abs() / size)
    o = omap[None]
    o = F.conv2d(F.pad(o, (size - 1, size - 1, 0, 0)), tri.view(1, 1, 1, -1).repeat(nori, 1, 1, 1), groups=nori)
    o = F.conv2d(F.pad(o, (0, 0, size - 1, size - 1)), tri.view(1, 1, -1, 1).repeat(nori, 1, 1, 1), groups=nori)
    o = o[0]                                       # [nori, H, W]: pooled histogram centred at each pixel
    # keypoint grid: the 4x4 bin centres must stay inside the image
    half = 2 * size
    ys = torch.arange(half - 1, H - half + 1, step, device=dev)
    xs = torch.arange(half - 1, W - half + 1, step, device=dev)
    if ys.numel() == 0 or xs.numel() == 0:
        return torch.zeros(2, 0, device=dev), torch.zeros(128, 0, device=dev)
    offs = (torch.arange(4, device=dev, dtype=dt) - 1.5) * size   # bin centres relative to the keypoint
    by = (ys[:, None].to(dt) + offs[None, :]).round().long().clamp(0, H - 1)    # [ny, 4]
    bx = (xs[:, None].to(dt) + offs[None, :]).round().long().clamp(0, W - 1)    # [nx, 4]
    d = o[:, by[:, None, :, None], bx[None, :, None, :]]                          # [nori, ny, nx, 4, 4]
    d = d.permute(1, 2, 3, 4, 0).reshape(ys.numel() * xs.numel(), 128)
    d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
    d = d.clamp(max=0.2)
    d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
    fy, fx = torch.meshgrid(ys, xs, indexing="ij")
    frames = torch.stack([fx.reshape(-1), fy.reshape(-1)]).to(dt)
    return frames, d.T


def root_sift(d: torch.Tensor) -> torch.Tensor:
    """RootSIFT (``relja_rootsift``): L1-normalise each column, then sqrt."""
    return torch.sqrt(d / d.abs().sum(0, keepdim=True).clamp_min(1e-12))


# ---------------------------------------------------------------------------
def pv_score(query_img: np.ndarray, rgb: np.ndarray, xyz: np.ndarray, P: np.ndarray, focal: float,
             device: str | torch.device = "cpu", ds: float = DS_LEVEL):
    """Dense-PV score of one pose candidate (parfor_nc4d_PV.m).

    query_img [H, W, 3] uint8/float (full resolution), rgb/xyz [N, 3] the scan
    (xyz already in the global frame), P [3, 4], focal in full-res pixels.
    Returns (score, synth_rgb [h, w, 3], valid mask [h, w], errmap [ny, nx]).
    """
    if P is None or not np.all(np.isfinite(P)):
        return 0.0, None, None, None
    dev = torch.device(device)
    q = torch.as_tensor(np.asarray(query_img, np.float32), device=dev)
    if q.ndim == 2:
        q = q[..., None].repeat(1, 1, 3)
    hq, wq = max(1, int(round(q.shape[0] * ds))), max(1, int(round(q.shape[1] * ds)))
    qs = F.interpolate(q.permute(2, 0, 1)[None], size=(hq, wq), mode="bilinear", align_corners=False,
                       antialias=True)[0].permute(1, 2, 0)
    fl = focal * ds
    K = torch.tensor([[fl, 0, wq / 2.0], [0, fl, hq / 2.0], [0, 0, 1]], dtype=torch.float64, device=dev)
    KP = K @ torch.as_tensor(np.asarray(P, np.float64), device=dev)
    rgb_t = torch.as_tensor(np.asarray(rgb, np.float32), device=dev)
    xyz_t = torch.as_tensor(np.asarray(xyz, np.float64), device=dev)
    synth, synth_xyz = points_to_perspective(rgb_t, xyz_t, KP, hq, wq)
    flag = ~torch.isnan(synth_xyz).any(-1)
    if not bool(flag.any()):
        return 0.0, synth.cpu().numpy(), flag.cpu().numpy(), None
    scale = 255.0 if float(qs.max()) > 1.5 else 1.0
    iq = image_normalization(rgb2gray(qs) / scale, flag)
    gs = rgb2gray(synth) / (255.0 if float(torch.nan_to_num(synth).max()) > 1.5 else 1.0)
    gs = torch.where(flag, gs, torch.full_like(gs, float("nan")))
    isyn = image_normalization(inpaint_nans(gs), flag)
    fq, dq = dense_sift(iq)
    fs, dsy = dense_sift(isyn)
    if fs.shape[1] == 0:
        return 0.0, synth.cpu().numpy(), flag.cpu().numpy(), None
    iseval = flag[fs[1].long(), fs[0].long()]
    dq, dsy = root_sift(dq), root_sift(dsy)
    err = torch.sqrt(((dq[:, iseval] - dsy[:, iseval]) ** 2).sum(0))
    if err.numel() == 0:
        return 0.0, synth.cpu().numpy(), flag.cpu().numpy(), None
    med = float(torch.quantile(err, 0.5))
    score = 1.0 / med if med > 0 else float("inf")
    errmap = torch.full((fs.shape[1],), float("nan"), device=dev)
    errmap[iseval] = err
    ny = int(torch.unique(fs[1]).numel())
    return score, synth.cpu().numpy(), flag.cpu().numpy(), errmap.view(ny, -1).cpu().numpy()


def rerank(candidates, scores):
    """Sort candidates (list of (dbname, P)) by PV score, descending
    (ht_top10_NC4D_PV_localization.m:63-67); stable for ties."""
    order = sorted(range(len(scores)), key=lambda i: -scores[i])
    return [candidates[i] for i in order], [scores[i] for i in order]


# ---------------------------------------------------------------------------
# InLoc scan I/O
_CUTOUT = re.compile(r"^(?P<floor>[^/]+)/(?P<scan>[^/]+)/(?P<scene>[A-Za-z0-9]+)_cutout_(?P<scan2>[^_]+)_.*$")


def parse_cutout_name(dbname: str):
    """``DUC1/024/DUC_cutout_024_30_0.jpg`` -> (floor, scene_id, scan_id)
    (InLoc_demo ``parse_WUSTL_cutoutname``; naming of the InLoc cutouts)."""
    m = _CUTOUT.match(dbname.replace("\\", "/"))
    if not m:
        raise ValueError(f"not an InLoc cutout name: {dbname}")
    return m.group("floor"), m.group("scene"), m.group("scan")


def scan_paths(dbname: str, scan_dir: str, scan_suffix: str = ".ptx.mat"):
    """Scan point cloud and its transformation file for a cutout
    (ht_top10_NC4D_PV_localization.m:24-27)."""
    floor, scene, scan = parse_cutout_name(dbname)
    return (os.path.join(scan_dir, floor, f"{scene}_scan_{scan}{scan_suffix}"),
            os.path.join(scan_dir, floor, "transformations", f"{scene}_trans_{scan}.txt"))


def load_transformation(path: str) -> np.ndarray:
    """4x4 scan-to-global matrix from an InLoc transformation text file: the
    last 4 rows of numbers (``load_WUSTL_transformation``'s P_after)."""
    rows = []
    with open(path) as f:
        for line in f:
            vals = line.replace(",", " ").split()
            try:
                nums = [float(v) for v in vals]
            except ValueError:
                continue
            if len(nums) == 4:
                rows.append(nums)
    if len(rows) < 4:
        raise ValueError(f"no 4x4 matrix in {path}")
    return np.asarray(rows[-4:], np.float64)


def load_scan(path: str, P_after: np.ndarray | None = None):
    """InLoc ``.ptx.mat`` scan: cell ``A`` with x, y, z, intensity, r, g, b
    columns (at_pv_wrapper.m:9-14) -> (rgb [N, 3], xyz [N, 3] global)."""
    from scipy.io import loadmat   # MATLAB v5 reader; executes nothing from the file

    A = loadmat(path)["A"].reshape(-1)
    xyz = np.stack([np.asarray(A[i], np.float64).reshape(-1) for i in range(3)], 1)
    rgb = np.stack([np.asarray(A[i], np.float64).reshape(-1) for i in (4, 5, 6)], 1)
    if P_after is not None:
        Xh = np.concatenate([xyz, np.ones((xyz.shape[0], 1))], 1) @ np.asarray(P_after, np.float64).T
        xyz = Xh[:, :3] / Xh[:, 3:4]
    return rgb, xyz
