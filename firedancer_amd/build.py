"""In-tree build of the native parts (run on the CPU build container; the
.so files travel to the GPU box with the snapshot).

* libfdgpu_ed25519.so -- HIP kernels + C-ABI runtime, hipcc for gfx950
* libfdsynth.so       -- host C synthetic-transaction generator
"""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
ARCH = os.environ.get("FDGPU_ARCH", "gfx950")

HIP_SRCS = ["fd_ed25519_gpu.hip"]
HIP_DEPS = ["fd_gpu_f25519.h", "fd_gpu_sha512.h", "fd_gpu_curve.h", "fd_gpu_txn.h", "fd_gpu_lattice.h",
            "../../include/fd_ed25519_gpu.h"]


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(os.path.join(CSRC, d)) > t for d in deps)


def build_engine(force: bool = False, extra: list[str] | None = None) -> str:
    out = os.path.join(PKG, "libfdgpu_ed25519.so")
    if force or extra or _stale(out, HIP_SRCS + HIP_DEPS):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result", "-o", out] + (extra or []) + [os.path.join(CSRC, s) for s in HIP_SRCS]
        subprocess.run(cmd, check=True, cwd=CSRC)
    return out


def build_synth(force: bool = False) -> str:
    out = os.path.join(PKG, "libfdsynth.so")
    if force or _stale(out, ["fd_synth.c", "../../include/fd_ed25519_gpu.h"]):
        subprocess.run(["gcc", "-std=gnu11", "-O2", "-fPIC", "-shared", "-pthread", "-o", out,
                        os.path.join(CSRC, "fd_synth.c")], check=True)
    return out


def build_vtile(force: bool = False) -> str:
    """libfdgpu_vtile.so: the verify tile and the verify service over the engine (host C, links libfdgpu_ed25519.so)."""
    out = os.path.join(PKG, "libfdgpu_vtile.so")
    eng = os.path.join(PKG, "libfdgpu_ed25519.so")
    if force or _stale(out, ["fd_verify_gpu.c", "fd_vsvc.c", "fd_vsvc_private.h", "../../include/fd_verify_gpu.h",
                             "../../include/fd_ed25519_gpu.h"]) \
            or os.path.getmtime(eng) > os.path.getmtime(out):
        subprocess.run(["gcc", "-std=gnu11", "-O2", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra",
                        "-o", out, os.path.join(CSRC, "fd_verify_gpu.c"), os.path.join(CSRC, "fd_vsvc.c"), eng,
                        "-Wl,-rpath,$ORIGIN"], check=True)
    return out


def build_tile_prog(force: bool = False) -> str:
    """fdgpu_tile: a served verify tile as a program of its own (fd_vtile_main.c over libfdgpu_vtile.so); the verify
    service's process starts one per tile (fdgpu_link_run with cfg.svc)."""
    out = os.path.join(PKG, "fdgpu_tile")
    lib = os.path.join(PKG, "libfdgpu_vtile.so")
    if force or _stale(out, ["fd_vtile_main.c", "../../include/fd_verify_gpu.h"]) or os.path.getmtime(lib) > os.path.getmtime(out):
        subprocess.run(["gcc", "-std=gnu11", "-O2", "-Wall", "-Wextra", "-o", out, os.path.join(CSRC, "fd_vtile_main.c"),
                        lib, "-Wl,-rpath,$ORIGIN"], check=True)
    return out


def build_lattice_host(force: bool = False) -> str:
    """libfdlat_host.so: the device half-size-scalar reduction (fd_gpu_lattice.h) compiled as host C,
    for tests/test_lattice.py only (the product calls it inside fd_hashh_kernel)."""
    out = os.path.join(PKG, "libfdlat_host.so")
    if force or _stale(out, ["fd_lat_host.c", "fd_gpu_lattice.h"]):
        subprocess.run(["gcc", "-std=gnu11", "-O2", "-Wall", "-Wno-unknown-pragmas", "-fPIC", "-shared", "-o", out,
                        os.path.join(CSRC, "fd_lat_host.c")], check=True)
    return out


def build_all(force: bool = False) -> None:
    build_synth(force)
    build_lattice_host(force)
    build_engine(force)
    build_vtile(force)
    build_tile_prog(force)


if __name__ == "__main__":
    build_all(force=True)
