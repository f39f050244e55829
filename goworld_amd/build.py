"""Build libgwaoi.so (hand-written HIP for gfx950) in-tree: goworld_amd/libgwaoi.so.

Called by __graft_entry__.build(); runnable as `python -m goworld_amd.build`. hipcc cross-compiles
for gfx950 without a GPU. IEEE binary32 semantics are part of the product's contract (bit-exact
AOI events), hence -ffp-contract=off and preserved denormals.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgwaoi.so")
SOURCES = ["gwaoi_kernels.hip", "gwaoi_runtime.hip", "gwaoi_strips.hip", "gwaoi_sync.hip", "gwaoi_comm.hip"]
HEADERS = ["gwaoi_internal.h"]
PUBLIC = ["gwaoi.h", "gwaoi_tools.h", "gwaoi_workload.h", "gwaoi_strips.h", "gwaoi_sync.h"]
ARCH = os.environ.get("GWAOI_ARCH", "gfx950")


def hipcc() -> str:
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if p and os.path.exists(p):
            return p
    return "hipcc"


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", f) for f in PUBLIC]
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps)


def source_hash(defines=()) -> str:
    """sha256 (16 hex digits) over the library's sources, headers, compile flags and A/B defines. It is
    compiled into the library (gwaoi_version() ends with "src <hash>") so that measurements taken with
    one build (the PMC traffic in profiles/pmc_latest.json) can be matched to the library bench.py loads."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(SOURCES + HEADERS + ["gwaoi_device.h"]):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    for f in sorted(PUBLIC):
        with open(os.path.join(ROOT, "include", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    h.update(" ".join(_FLAGS + [f"-D{d}" for d in defines] + [ARCH]).encode())
    return h.hexdigest()[:16]


_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
          "-fno-gpu-flush-denormals-to-zero", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Compile the library to `out`; `defines` (e.g. ["GW_SWEEP_BLOCK=512"]) builds an A/B variant."""
    if not force and out == OUT and not _stale():
        return OUT
    # _FLAGS: IEEE binary32 (no contraction, denormals kept); LDS event-queue atomics are one
    # ds_add_rtn each (the wave-reduction rewrite the atomic optimizer wraps around every call costs
    # more than it saves at ~1 event per 100 candidates)
    cmd = [
        hipcc(), f"--offload-arch={ARCH}", *_FLAGS, f'-DGWAOI_SRC_HASH="{source_hash(defines)}"',
        "-Wall", "-Wno-unused-result", "-Wno-unused-value",
        f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}",
        *[f"-D{d}" for d in defines],
        *[os.path.join(CSRC, f) for f in SOURCES],
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib",  # the X-strip halo exchange (gwaoi_comm.hip)
        "-o", out + ".tmp",
    ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
