"""Compiler resource usage of every gfx950 kernel in ``csrc/*.hip``.

Runs hipcc with ``-Rpass-analysis=kernel-resource-usage`` (device code only,
no link) and parses its remarks into one record per kernel instantiation:
VGPRs, AGPRs, SGPRs, scratch bytes per lane, spilled VGPRs/SGPRs, occupancy
(waves per SIMD) and static LDS.  ``tests/test_kernel_resources.py`` uses it to
fail the CPU suite when a hot kernel starts spilling (the round-2 regression:
conv16v3 fwd/dgrad picked up scratch from a release-mode codegen change).

    python -m ncnet_amd.kernel_resources [--md out.md] [file.hip ...]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import re
import subprocess
import sys
from pathlib import Path

from .build import CSRC, HIP_FLAGS, HIPCC, resource_cache, resource_key

_FIELDS = {
    "VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
    "Occupancy [waves/SIMD]": "occupancy", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
    "LDS Size [bytes/block]": "lds",
}
_REMARK = re.compile(r"remark: ([^:]+(?: \[[^\]]*\])?): (.*?) \[-Rpass-analysis=kernel-resource-usage\]")


def demangle(name: str) -> str:
    """Readable kernel name: the compiler prints templates in namespace
    ``ncnet`` mangled (bf16 parameters defeat c++filt), so decode the
    identifier and its integer/bool template arguments by hand."""
    m = re.match(r"_ZN5ncnet(\d+)", name)
    if not m:
        return name
    n = int(m.group(1))
    start = m.end()
    ident = name[start:start + n]
    rest = name[start + n:]
    if rest.startswith("I"):
        args = re.findall(r"L([ib])(\d+)E", rest[:rest.find("EE") + 2])
        vals = [("true" if v == "1" else "false") if t == "b" else v for t, v in args]
        return f"{ident}<{', '.join(vals)}>"
    return ident


def _cached_remarks(src: Path) -> str | None:
    """The remarks the release build wrote for ``src`` (ncnet_amd/build.py), if
    they were produced from this exact source, headers and flags."""
    path = resource_cache(src)
    if not path.exists():
        return None
    text = path.read_text()
    first, _, rest = text.partition("\n")
    return rest if first == f"# key {resource_key(src)}" else None


def analyse(src: Path, extra_flags=(), use_cache: bool = True) -> list[dict]:
    """Resource records of every kernel compiled from ``src`` (from the build's
    remarks when they match the source, else a device-only compile)."""
    src = Path(src)
    text = _cached_remarks(src) if use_cache and not extra_flags else None
    if text is None:
        flags = [f for f in HIP_FLAGS if f != "-fPIC"]
        cmd = [HIPCC, *flags, *extra_flags, "-I", str(CSRC), "--offload-device-only", "-c", str(src), "-o",
               "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-4000:]}")
        text = r.stderr
    recs, cur = [], None
    for line in text.splitlines():
        m = _REMARK.search(line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"file": src.name, "mangled": val}
            recs.append(cur)
        elif cur is not None and key in _FIELDS:
            try:
                cur[_FIELDS[key]] = int(val)
            except ValueError:
                cur[_FIELDS[key]] = val
    for rec in recs:
        rec["name"] = demangle(rec["mangled"])
    return recs


def analyse_all(srcs=None, jobs: int = 4) -> list[dict]:
    srcs = [Path(s) for s in srcs] if srcs else sorted(CSRC.glob("*.hip"))
    # largest (slowest) sources first so the long compiles overlap the short ones
    order = sorted(range(len(srcs)), key=lambda i: -srcs[i].stat().st_size)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {i: ex.submit(analyse, srcs[i]) for i in order}
        return [rec for i in range(len(srcs)) for rec in futs[i].result()]


def short(name: str) -> str:
    """'ncnet::conv16v3_fwd_kernel<5, 5, 1>(...)' -> 'conv16v3_fwd_kernel<5, 5, 1>'."""
    s = name.split("(")[0]
    return s.replace("ncnet::", "").replace("void ", "")


def to_markdown(recs) -> str:
    lines = ["| kernel | file | VGPR | AGPR | SGPR | scratch B/lane | VGPR spill | SGPR spill | waves/SIMD |",
             "|---|---|---:|---:|---:|---:|---:|---:|---:|"]
    for r in recs:
        lines.append(f"| `{short(r.get('name', r['mangled']))}` | {r['file']} | {r.get('vgpr', '')} | {r.get('agpr', '')} "
                     f"| {r.get('sgpr', '')} | {r.get('scratch', '')} | {r.get('vgpr_spill', '')} "
                     f"| {r.get('sgpr_spill', '')} | {r.get('occupancy', '')} |")
    return "\n".join(lines) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("srcs", nargs="*")
    ap.add_argument("--md", default=None, help="write a markdown table here")
    a = ap.parse_args(argv)
    recs = analyse_all(a.srcs)
    md = to_markdown(recs)
    if a.md:
        Path(a.md).write_text(md)
    print(md)
    bad = [r for r in recs if r.get("scratch", 0) or r.get("vgpr_spill", 0)]
    print(f"{len(recs)} kernels, {len(bad)} with scratch / VGPR spills")


if __name__ == "__main__":
    sys.exit(main())
