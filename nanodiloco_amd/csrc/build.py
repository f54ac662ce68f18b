"""Build the native libraries in-tree (no JIT cache, no hipify, no torch headers).

  nanodiloco_amd/_lib/libnd_kernels.so   every csrc/*.hip, hipcc --offload-arch=gfx950 -O3
  nanodiloco_amd/_lib/libnd_runtime.so   csrc/runtime/*.cpp (host C++: token loader), g++ -O3
  nanodiloco_amd/_lib/libnd_comm.so      csrc/comm/*.cpp (host C++: own RCCL communicator), hipcc -lrccl

Usage:  python -m nanodiloco_amd.csrc.build [--force] [--jobs N] [--save-temps]
Incremental: an object is rebuilt only when the content hash of its source / headers / flags changed.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shlex
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_DIR = os.path.join(PKG, "_lib")
OBJ_DIR = os.path.join(PKG, "_lib", "obj")
ARCH = os.environ.get("ND_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError("hipcc not found (ROCm >= 7 required)")


def _digest(files, extra="") -> str:
    h = hashlib.sha256(extra.encode())
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale(src_files, target, extra="") -> bool:
    """Content-hash staleness (mtimes do not survive snapshot copies to the GPU box)."""
    stamp = target + ".sha256"
    if not os.path.exists(target) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(src_files, extra)


def _mark(src_files, target, extra=""):
    with open(target + ".sha256", "w") as f:
        f.write(_digest(src_files, extra))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


# Per-file extra flags.  attention.hip: no SLP vectorisation -- packed f32 VALU (v_pk_mul_f32 /
# v_pk_fma_f32) issued beside MFMAs costs more than two scalar ops (MI355X_MICROARCH price list).
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"],
              # gemm_w128.hip: its phases are 64-slot loops that must unroll completely (every
              # accumulator index a constant); past the default pragma threshold the accumulator array
              # silently moves to scratch
              "gemm_w128.hip": ["-mllvm", "-pragma-unroll-threshold=1000000"]}


def build(force: bool = False, jobs: int = 0, save_temps: bool = False, verbose: bool = False) -> dict:
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = _hipcc()
    headers = glob.glob(os.path.join(HERE, "*.h"))
    sources = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-I", HERE]
    flags += shlex.split(os.environ.get("ND_EXTRA_HIPCC_FLAGS", ""))  # A/B or ablation builds only
    if save_temps:
        flags += ["-save-temps"]
    kern = os.path.join(LIB_DIR, "libnd_kernels.so")
    # fast path: the library was linked from exactly these sources / headers / flags (object files do
    # not travel to the GPU box, so without this every fresh checkout would recompile everything)
    src_key = " ".join(flags) + repr(sorted(FILE_FLAGS.items()))
    src_stamp = kern + ".src.sha256"
    all_src = sources + sorted(headers)
    if not force and os.path.exists(kern) and os.path.exists(src_stamp):
        with open(src_stamp) as f:
            if f.read().strip() == _digest(all_src, src_key):
                return _build_runtime(force, kern, [])
    todo = []
    objs = []
    for s in sources:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale([s] + sorted(headers), o, " ".join(flags + FILE_FLAGS.get(os.path.basename(s), []))):
            todo.append((s, o))
    # objects of sources that no longer exist (renamed / removed kernels) are deleted, never linked
    for o in glob.glob(os.path.join(OBJ_DIR, "*.hip.o")):
        if o not in objs:
            for f in (o, o + ".sha256"):
                if os.path.exists(f):
                    os.remove(f)
    jobs = jobs or min(8, os.cpu_count() or 4)

    def comp(so):
        s, o = so
        cwd = OBJ_DIR if save_temps else None
        fl = flags + FILE_FLAGS.get(os.path.basename(s), [])
        r = subprocess.run([hipcc] + fl + ["-c", s, "-o", o], capture_output=True, text=True, cwd=cwd)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {os.path.basename(s)}:\n{r.stderr[-6000:]}")
        _mark([s] + sorted(headers), o, " ".join(fl))
        return s

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in ex.map(comp, todo):
            if verbose:
                print(f"[build] compiled {os.path.basename(s)}", flush=True)
    if force or todo or _stale(objs, kern):
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", kern + ".tmp"] + objs)
        os.replace(kern + ".tmp", kern)
        _mark(objs, kern)
    with open(src_stamp, "w") as f:
        f.write(_digest(all_src, src_key))
    return _build_runtime(force, kern, todo)


def _build_runtime(force, kern, todo) -> dict:
    # host runtime (plain C++)
    rt_src = sorted(glob.glob(os.path.join(HERE, "runtime", "*.cpp")))
    rt = os.path.join(LIB_DIR, "libnd_runtime.so")
    if rt_src and (force or _stale(rt_src, rt)):
        cxx = shutil.which("g++") or shutil.which("c++")
        _run([cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", rt + ".tmp"] + rt_src)
        os.replace(rt + ".tmp", rt)
        _mark(rt_src, rt)
    # own RCCL communicator (host code against librccl / the HIP runtime; no device code)
    cm_src = sorted(glob.glob(os.path.join(HERE, "comm", "*.cpp")))
    cm = os.path.join(LIB_DIR, "libnd_comm.so")
    if cm_src and (force or _stale(cm_src, cm)):
        _run([_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", cm + ".tmp"] + cm_src + ["-lrccl"])
        os.replace(cm + ".tmp", cm)
        _mark(cm_src, cm)
    return {"kernels": kern, "runtime": rt, "comm": cm, "compiled": [os.path.basename(s) for s, _ in todo]}


def build_ablation(jobs: int = 0) -> str:
    """The timing-ablation library: the working tree's csrc/ with -DND_ABLATION, which compiles in the
    kernel variants that skip loads / barriers / MFMAs / stores (WRONG results, profiling only) into
    _lib/alt/libnd_kernels_ablation.so.  The product library never contains them; load this one with
    ND_KERNELS_LIB=<path> (ops/_ext.py) or ``_ext.load_library`` in the ablation scripts."""
    return build_revision(None, jobs, ["-DND_ABLATION=1"], tag="ablation")


def build_revision(rev, jobs: int = 0, extra_flags=None, file_flags: bool = True, tag: str = "") -> str:
    """Build libnd_kernels.so from the csrc/ of git revision `rev` (None: the working tree) into _lib/alt/
    (for in-process A/B against the working tree: device-to-device and run-to-run variance on MI355X is
    several percent, so code versions are compared interleaved inside one process; see scripts/ab_kernels.py)."""
    import tempfile
    root = os.path.dirname(PKG)
    if rev is None:
        srcs_wt = sorted(glob.glob(os.path.join(HERE, "*.hip")) + glob.glob(os.path.join(HERE, "*.h")))
        out = os.path.join(LIB_DIR, "alt", f"libnd_kernels_{tag or 'wt'}.so")
        key = _digest(srcs_wt, " ".join(extra_flags or []))
        if os.path.exists(out) and not _stale(srcs_wt, out, " ".join(extra_flags or [])):
            return out
    else:
        sha = _run(["git", "-C", root, "rev-parse", "--short", rev]).stdout.strip()
        out = os.path.join(LIB_DIR, "alt", f"libnd_kernels_{sha}{('_' + tag) if tag else ''}.so")
        if os.path.exists(out):
            return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = _hipcc()
    with tempfile.TemporaryDirectory() as td:
        if rev is None:
            srcs = []
            for n in srcs_wt:
                dst = os.path.join(td, os.path.basename(n))
                shutil.copyfile(n, dst)
                if n.endswith(".hip"):
                    srcs.append(dst)
        else:
            names = _run(["git", "-C", root, "ls-tree", "--name-only", rev, "nanodiloco_amd/csrc/"]).stdout.split()
            srcs = []
            for n in names:
                if n.endswith((".hip", ".h")):
                    dst = os.path.join(td, os.path.basename(n))
                    with open(dst, "w") as f:
                        f.write(_run(["git", "-C", root, "show", f"{rev}:{n}"]).stdout)
                    if n.endswith(".hip"):
                        srcs.append(dst)
        flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-I", td]
        flags += list(extra_flags or [])

        def comp(src):
            o = src + ".o"
            ff = FILE_FLAGS.get(os.path.basename(src), []) if file_flags else []
            _run([hipcc] + flags + ff + ["-c", src, "-o", o])
            return o

        with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
            objs = list(ex.map(comp, srcs))
        # -Bsymbolic: the side library's references to its own kernel stubs must not bind to the
        # identically named symbols of the main library already loaded RTLD_GLOBAL
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-Bsymbolic", "-o", out] + objs)
    if rev is None:
        with open(out + ".sha256", "w") as f:
            f.write(key)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--save-temps", action="store_true")
    ap.add_argument("--rev", default=None, help="build the kernels of this git revision into _lib/alt/ (A/B)")
    ap.add_argument("--extra-flags", default="", help="with --rev: extra hipcc flags (compiler-option A/B)")
    ap.add_argument("--no-file-flags", action="store_true", help="with --rev: drop the per-file flags")
    ap.add_argument("--tag", default="", help="with --rev: suffix of the side library's file name")
    ap.add_argument("--ablation", action="store_true",
                    help="build the timing-ablation library (-DND_ABLATION, wrong-result variants) into _lib/alt/")
    a = ap.parse_args(argv)
    if a.ablation:
        print(build_ablation(a.jobs))
        return
    if a.rev:
        # --rev WT: the working tree (uncommitted edits) into _lib/alt/libnd_kernels_<tag>.so
        rev = None if a.rev == "WT" else a.rev
        print(build_revision(rev, a.jobs, a.extra_flags.split(), not a.no_file_flags, a.tag))
        return
    out = build(force=a.force, jobs=a.jobs, save_temps=a.save_temps, verbose=True)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
