"""InLoc dense-match export (eval_inloc.py), with the same ``.mat`` contract.

Per query: ``matches`` float64 ``[1, n_panos, N, 5]`` with columns
``(xA, yA, xB, yB, score)`` in pixel-centre-normalised [0,1] coordinates,
unused rows 0, plus ``query_fn`` and ``pano_fn`` (eval_inloc.py:126,197-221).

Differences from the reference, output-preserving:
* the bidirectional de-duplication (sort by score, ``np.unique`` on the CPU,
  eval_inloc.py:160-173) runs on the GPU with integer keys: the kept match of
  every (xA,yA,xB,yB) is the highest-scoring one and the rows come out in the
  lexicographic (xA,yA,xB,yB) order that ``np.unique`` produces;
* query files that already exist are skipped (resume by idempotence, the same
  idea as the MATLAB stage caching), and queries can be sharded over ranks.
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch

from .. import config as _config
from ..data.transforms import normalize_image, resize_bilinear
from ..ops.neigh_consensus import pin_fp8_weights
from ..ops import _ext
from .point_tnf import best_both, corr_to_matches

SCALE_FACTOR = 0.0625  # feature stride 1/16 (eval_inloc.py:77)
# MIOpen solver search (torch.backends.cudnn.benchmark) of the InLoc runs:
# eval_inloc.py and bench.py's InLoc secondaries both run in this state, so the
# bench times the trunk kernels the CLI runs (3200 px bf16 measured 10.6-10.8
# ms/pair with it off or on, profiles/r5/inloc/cudnn_ab.txt)
INLOC_CUDNN_BENCHMARK = False


def output_folder(shortlist: str, image_size: int, k_size: int, both_dirs: bool, flip: bool, softmax: bool,
                  checkpoint: str = "") -> str:
    """eval_inloc.py:60-71."""
    name = os.path.basename(shortlist).split(".")[0] + "_SZ_NEW_" + str(image_size) + "_K_" + str(k_size)
    if both_dirs:
        name += "_BOTHDIRS"
    elif flip:
        name += "_AtoB"
    else:
        name += "_BtoA"
    if softmax:
        name += "_SOFTMAX"
    if checkpoint:
        name += "_CHECKPOINT_" + os.path.basename(checkpoint).split(".")[0]
    return name


def n_matches(image_size: int, k_size: int, both_dirs: bool) -> int:
    """eval_inloc.py:116-118 (sized for 4:3 landscape images)."""
    a = image_size * SCALE_FACTOR / k_size
    n = int(a * np.floor(a * 3 / 4))
    return 2 * n if both_dirs else n


def target_size(h: int, w: int, image_size: int, k_size: int):
    """Longest side -> image_size, floored to a multiple of k_size/0.0625 px
    when relocalizing (eval_inloc.py:83-89)."""
    r = max(h, w) / image_size
    if k_size == 1:
        return int(h / r), int(w / r)
    unit = SCALE_FACTOR / k_size
    return (int(np.floor(h / r * unit) / unit), int(np.floor(w / r * unit) / unit))


def prepare_image(img_uint8_hwc: np.ndarray, image_size: int, k_size: int, device) -> torch.Tensor:
    x = torch.from_numpy(np.ascontiguousarray(img_uint8_hwc.transpose(2, 0, 1))).to(device).float() / 255.0
    x = normalize_image(x)
    h, w = target_size(x.shape[1], x.shape[2], image_size, k_size)
    return resize_bilinear(x, h, w).unsqueeze(0)


def _fused_candidates(corr4d, delta4d, k: int, do_softmax: bool):
    """Both directions' match candidates of a single volume in two HIP launches
    (stats2d + match_candidates: the ~60 small index / gather / arithmetic ops
    of two corr_to_matches calls, their concatenation and the recentre) ->
    (m [N, 5] recentred, sc [N], key [N] int64) in the same order and values as
    the op-by-op path, or None where it does not apply."""
    b, _, fs1, fs2, fs3, fs4 = corr4d.shape
    if b != 1 or not (_ext.use_hip(corr4d) and corr4d.dtype == torch.float32):
        return None
    if delta4d is not None and k > 4:
        # the kernel decodes 2-bit offsets: k_size > 4 stays on the op-by-op path
        return None
    if delta4d is not None and not torch.is_tensor(delta4d):
        # unpacked (di, dj, dk, dl) offsets -> the packed 2-bit code (same decode as the fused pool's codes)
        if len(delta4d) != 4:
            return None
        d = [t.reshape(-1).to(torch.int32) for t in delta4d]
        delta4d = ((d[0] << 6) | (d[1] << 4) | (d[2] << 2) | d[3]).to(torch.uint8)
    elif delta4d is not None and delta4d.dtype != torch.uint8:
        return None
    R, C = fs1 * fs2, fs3 * fs4
    x = corr4d.reshape(1, R, C).contiguous()
    dev = x.device
    f = dict(dtype=torch.float32, device=dev)
    rmx, cmx = torch.empty((1, R), **f), torch.empty((1, C), **f)
    rarg = torch.empty((1, R), dtype=torch.int32, device=dev)
    carg = torch.empty((1, C), dtype=torch.int32, device=dev)
    rse = torch.empty((1, R), **f) if do_softmax else None
    cse = torch.empty((1, C), **f) if do_softmax else None
    E = _ext.ext()
    if not E.stats2d(x, rmx, rarg, rse, cmx, carg, cse, 1 if do_softmax else 0):
        return None
    m = torch.empty((R + C, 5), **f)
    sc = torch.empty((R + C,), **f)
    key = torch.empty((R + C,), dtype=torch.int64, device=dev)
    code = delta4d.reshape(-1) if delta4d is not None else None
    E.match_candidates(cmx[0], cse[0] if do_softmax else None, carg[0], rmx[0], rse[0] if do_softmax else None,
                       rarg[0], code, fs1, fs2, fs3, fs4, k, m, sc, key)
    return m, sc, key


def _dedup(sc, key):
    """Stable de-duplication order: by score (descending), then by key; the
    first of equal keys is kept -> (idx, first)."""
    order = torch.argsort(-sc, stable=True)
    key_s = key[order]
    order2 = torch.argsort(key_s, stable=True)
    idx = order[order2]
    ks_ = key[idx]
    first = torch.ones_like(ks_, dtype=torch.bool)
    first[1:] = ks_[1:] != ks_[:-1]
    return idx, first


def pair_matches(corr4d, delta4d, k_size: int, do_softmax: bool = True, both_dirs: bool = True,
                 flip: bool = False, static: bool = False):
    """Bidirectional, de-duplicated, recentred matches of one pair -> [Npts, 5] tensor.

    ``static``: shapes independent of the data (HIP-graph capturable): returns
    ``(out [M, 5], count)`` with the ``count`` unique matches in the same order
    in the first rows and zeros after them (M = all candidate matches)."""
    b, _, fs1, fs2, fs3, fs4 = corr4d.shape
    k = max(1, k_size)
    kw = dict(scale="positive", do_softmax=do_softmax, delta4d=delta4d, k_size=k, return_indices=True)
    if both_dirs:
        fc = _fused_candidates(corr4d, delta4d, k, do_softmax)
        if fc is not None:
            m_all, sc, key = fc
            idx, first = _dedup(sc, key)
            if static:
                pos = torch.cumsum(first.to(torch.int64), 0) - 1
                dst = torch.where(first, pos, torch.full_like(pos, idx.numel()))
                out = torch.zeros((idx.numel() + 1, 5), dtype=m_all.dtype, device=m_all.device)
                out.index_copy_(0, dst, m_all[idx])
                return out[:-1], first.sum()
            return m_all[idx[first]]
        both = best_both(corr4d, do_softmax)            # one pass for both directions where it applies
        r1 = corr_to_matches(corr4d, best=both[0] if both else None, **kw)
        r2 = corr_to_matches(corr4d, invert_matching_direction=True, best=both[1] if both else None, **kw)
        xA, yA, xB, yB, sc, iA, jA, iB, jB = (torch.cat((a.reshape(-1), c.reshape(-1))) for a, c in zip(r1, r2))
        HA, WA, HB, WB = fs1 * k, fs2 * k, fs3 * k, fs4 * k
        key = ((jA.long() * HA + iA.long()) * WB + jB.long()) * HB + iB.long()  # lexicographic (xA,yA,xB,yB)
        order = torch.argsort(-sc, stable=True)
        key_s = key[order]
        order2 = torch.argsort(key_s, stable=True)
        idx = order[order2]
        ks_ = key[idx]
        first = torch.ones_like(ks_, dtype=torch.bool)
        first[1:] = ks_[1:] != ks_[:-1]
        if static:
            # stable compaction without a data-dependent size: the kept rows go
            # to their rank among the kept, the duplicates to a dump row
            pos = torch.cumsum(first.to(torch.int64), 0) - 1
            dst = torch.where(first, pos, torch.full_like(pos, idx.numel()))
            m = _recentre(xA[idx], yA[idx], xB[idx], yB[idx], sc[idx], fs1, fs2, fs3, fs4, k)
            out = torch.zeros((idx.numel() + 1, 5), dtype=m.dtype, device=m.device)
            out.index_copy_(0, dst, m)
            return out[:-1], first.sum()
        idx = idx[first]
        xA, yA, xB, yB, sc = xA[idx], yA[idx], xB[idx], yB[idx], sc[idx]
    else:
        xA, yA, xB, yB, sc, *_ = corr_to_matches(corr4d, invert_matching_direction=flip, **kw)
        xA, yA, xB, yB, sc = (t.reshape(-1) for t in (xA, yA, xB, yB, sc))
    m = _recentre(xA, yA, xB, yB, sc, fs1, fs2, fs3, fs4, k)
    if static:
        return m, torch.tensor(m.shape[0], device=m.device)
    return m


def _recentre(xA, yA, xB, yB, sc, fs1, fs2, fs3, fs4, k):
    """Recentre to pixel centres (eval_inloc.py:180-189) -> [N, 5]."""
    n1, n2, n3, n4 = fs1 * k, fs2 * k, fs3 * k, fs4 * k
    yA = yA * (n1 - 1) / n1 + 0.5 / n1
    xA = xA * (n2 - 1) / n2 + 0.5 / n2
    yB = yB * (n3 - 1) / n3 + 0.5 / n3
    xB = xB * (n4 - 1) / n4 + 0.5 / n4
    return torch.stack((xA, yA, xB, yB, sc.float()), dim=1)


class PairMatcher:
    """Everything after the backbones for one query/pano pair -- correlation
    (+ k x k pool), MutualMatching, NeighConsensus, MutualMatching and the
    bidirectional de-duplicated match extraction -- replayed as one HIP graph
    per input shape (the ~60 launches of a pair otherwise leave gaps between
    the memory-bound kernels).  The graph is captured after two eager runs;
    if capture fails the matcher stays eager.  The returned tensors are
    reused by the next call: consume them first (eval_inloc.py copies them to
    the host)."""

    def __init__(self, model, k_size: int, do_softmax: bool = True, both_dirs: bool = True, flip: bool = False,
                 use_graph: bool | None = None):
        self.model, self.k = model, k_size
        self.kw = dict(do_softmax=do_softmax, both_dirs=both_dirs, flip=flip)
        self.use_graph = _config.RUNTIME.pair_graph if use_graph is None else use_graph
        self._graphs = {}
        self._nc_params = None
        self.capture_error = None
        self._last_fa = self._last_sa = None

    @property
    def graphed(self) -> bool:
        """True when at least one pair graph was captured and no capture failed."""
        return bool(self._graphs) and self.capture_error is None

    def _eager(self, fa, hwa, fb, hwb):
        out = self.model.match_features(fa, hwa, fb, hwb, packed_offsets=True)
        corr4d, delta = out if self.k > 1 else (out, None)
        return pair_matches(corr4d, delta, self.k, static=True, **self.kw)

    def __call__(self, fa, hwa, fb, hwb):
        if not (self.use_graph and torch.is_tensor(fa) and fa.is_cuda):
            return self._eager(fa, hwa, fb, hwb)
        # the graph bakes in the NC weights it was captured with (e.g. the
        # cached fp8 quantisation): a weight update must re-capture
        # (only the NeighConsensus weights enter the graph; ~6 tensors, cheap per pair)
        if self._nc_params is None:
            self._nc_params = list(self.model.NeighConsensus.parameters())
        wver = tuple(0 if p.is_inference() else p._version for p in self._nc_params)
        key = (tuple(fa.shape), tuple(fb.shape), fa.dtype, tuple(hwa), tuple(hwb), wver)
        ent = self._graphs.get(key)
        if ent is None:
            try:
                sa, sb = fa.clone(), fb.clone()
                side = torch.cuda.Stream(device=fa.device)
                side.wait_stream(torch.cuda.current_stream(fa.device))
                with torch.cuda.stream(side):
                    for _ in range(2):
                        self._eager(sa, hwa, sb, hwb)
                torch.cuda.current_stream(fa.device).wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with pin_fp8_weights() as pins, torch.cuda.graph(g):
                    res = self._eager(sa, hwa, sb, hwb)
                # stale shapes / weight versions are dropped with their graphs;
                # `pins` keeps the cached weight buffers the graph reads alive
                self._graphs = {k: v for k, v in self._graphs.items() if k[:5] != key[:5]}
                ent = self._graphs[key] = (g, sa, sb, res, pins)
            except RuntimeError as err:      # capture unsupported -> eager from now on (loudly)
                import traceback
                import warnings
                self.capture_error = "".join(traceback.format_exception(type(err), err, err.__traceback__))
                warnings.warn(f"PairMatcher: HIP graph capture disabled ({err})")
                self.use_graph = False
                return self._eager(fa, hwa, fb, hwb)
        g, sa, sb, res, _ = ent
        # a query's features are matched against its 10 panos: skip re-copying
        # the same (live) tensor object into the graph input (features are
        # not modified in place between calls)
        last = self._last_fa() if self._last_fa is not None else None
        if sa.data_ptr() != fa.data_ptr() and not (last is fa and self._last_sa is sa):
            sa.copy_(fa)
        self._last_fa, self._last_sa = weakref.ref(fa), sa
        sb.copy_(fb)
        g.replay()
        return res


def save_query(path: str, matches: np.ndarray, query_fn, pano_fns):
    from scipy.io import savemat

    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp.mat"
    savemat(tmp, {"matches": matches, "query_fn": query_fn, "pano_fn": pano_fns}, do_compression=True)
    os.replace(tmp, path)


def load_shortlist(path: str):
    """ImgList struct array -> (query names, [pano name lists])."""
    from scipy.io import loadmat

    db = loadmat(path)["ImgList"][0, :]
    queries = [str(np.asarray(db[q][0]).item()) for q in range(len(db))]
    panos = [[str(np.asarray(p).item()) for p in np.asarray(db[q][1]).ravel()] for q in range(len(db))]
    pano_all = np.vstack(tuple(np.asarray(db[q][1]) for q in range(len(db))))
    return queries, panos, pano_all
