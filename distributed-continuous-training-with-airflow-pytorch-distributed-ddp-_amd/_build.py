"""Build the native extension ``_dct_native`` in-tree with hipcc for gfx950.

No hipify, no torch.utils.cpp_extension (which would run hipify over the sources): every
``csrc/*.hip`` / ``csrc/*.cpp`` is compiled by ``hipcc --offload-arch=gfx950`` into
``build/obj`` (incremental on source/header mtimes + flags) and linked into
``<package>/_dct_native<EXT_SUFFIX>`` next to this file, so the built ``.so`` travels with
the repository snapshot to the GPU box.  ``python -m dct_amd._build`` builds it by hand.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(os.path.dirname(PKG_DIR), "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DCT_OFFLOAD_ARCH", "gfx950")
MODULE = "_dct_native"


def target_path() -> str:
    return os.path.join(PKG_DIR, MODULE + sysconfig.get_config_var("EXT_SUFFIX"))


# per-source extra flags.  The 3x128 trainers: the SLP vectorizer packs their independent fp32
# FMAs into v_pk_fma_f32 plus the v_mov_b32 pairs that marshal their operands - on gfx950 a packed op
# issues no faster than two plain ones, so the moves are pure overhead in an issue-bound kernel
# (mlp_block5 packs its Adam pairs by hand where packing pays).
# mlp_block5.hip (the one-rank 3x128 launches, the bench headline) also takes the max-ILP machine
# scheduler: 3.90 -> 3.80 us/step; its data-parallel unit keeps the default scheduler, under which
# the 8-rank kernels ran faster (12.85 vs 13.12 us/step, profiles/b5_sched_strategy_ab_r4.log).
# The TabTransformer block / io kernels too (VALU-issue bound: TT step 366 -> 356 us with them, the
# GEMM and skinny units under the same strategy made the tabular step 1 % slower; b5_sched_strategy_ab_r4.log).
# And the one-rank units of the 5-64-2 wave trainer: 0.640 / 0.655 -> 0.632 / 0.647 us/step long run,
# 20-step window 1.65-1.70 -> 1.60-1.69; its exchange units measured no gain at 2 / 4 ranks sharing a GPU
# (1.81 / 2.47 vs 1.80 / 2.47 us/step) and keep the default (profiles/wave_sched_strategy_ab_r4.log).
MAX_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
FILE_FLAGS = {"gemm_bf16.hip": ["-fno-slp-vectorize"],
              "optim.hip": ["-fno-slp-vectorize"],
              "mlp_block3.hip": ["-fno-slp-vectorize"],
              "mlp_block5.hip": ["-fno-slp-vectorize"] + MAX_ILP,
              "mlp_block5_xg.hip": ["-fno-slp-vectorize"],
              "mlp_block5_xgprof.hip": ["-fno-slp-vectorize"],
              "mlp_block5_b8.hip": ["-fno-slp-vectorize"],
              "mlp_block5_xgs.hip": ["-fno-slp-vectorize"],
              "tt_block.hip": MAX_ILP,
              "tt_io.hip": MAX_ILP,
              "mlp_wave_single.hip": MAX_ILP,
              "mlp_wave_rows_x0.hip": MAX_ILP}


def _sources():
    return sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp"))
    )


def _headers():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))


def _flags(debug: bool = False, sanitize: bool = None):
    import pybind11

    f = [
        f"--offload-arch={ARCH}",
        "-O0" if debug else "-O3",
        "-fPIC",
        "-std=c++17",
        "-Wno-unused-result",
        "-Wno-unused-variable",
        f"-I{CSRC}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        f"-I{ROCM}/include",
    ]
    if debug:
        f.append("-g")
    if os.environ.get("DCT_PROF_BUILD", "0") == "1":  # in-kernel phase stamps (tools/prof_fused.py)
        f.append("-DWAVE_PROF_BUILD")
    if sanitize is None:
        sanitize = os.environ.get("DCT_SANITIZE", "0") == "1"
    if sanitize:  # host-side ASan only (no GPU sanitizer on this pool)
        f += ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    return f


def _file_flags(base: str):
    """FILE_FLAGS of one source, plus the A/B-build flags (tools/so_ab.sh variants): AB_HIPCC_FLAGS
    (e.g. "-DB5_PRO=0") on the sources named in AB_HIPCC_FILES (comma-separated basenames)."""
    extra = []
    if base in os.environ.get("AB_HIPCC_FILES", "").split(","):
        extra = os.environ.get("AB_HIPCC_FLAGS", "").split()
    return FILE_FLAGS.get(base, []) + extra


def _stamp(src: str, flags) -> str:
    flags = list(flags) + _file_flags(os.path.basename(src))
    h = hashlib.sha1()
    h.update(" ".join(flags).encode())
    for p in [src] + _headers():
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _compile(src: str, flags, verbose: bool):
    os.makedirs(BUILD, exist_ok=True)
    base = os.path.basename(src)
    stamp = _stamp(src, flags)
    obj = os.path.join(BUILD, f"{base}.{stamp}.o")
    if os.path.exists(obj):
        return obj, False
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    tmp = f"{obj}.{os.getpid()}.tmp"  # per-process: concurrent builds never share a temp file
    cmd = [os.path.join(ROCM, "bin", "hipcc")] + flags + _file_flags(base) + lang + ["-c", src, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {base}:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, obj)
    return obj, True


def _manifest_path() -> str:
    return target_path() + ".objs"


def build(force: bool = False, verbose: bool = False, jobs: int = 0, debug: bool = False) -> str:
    """Compile what changed and relink when the linked object set differs from the current one.

    The object cache is keyed by source + header content and flags, so reverting a source finds
    its old object already built: the relink decision compares the object list recorded next to
    the .so (``<so>.objs``), not just "was anything recompiled".  Builds from several processes
    (torchrun ranks finding a stale extension) are serialised by a lock file."""
    import fcntl

    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        flags = _flags(debug)
        srcs = _sources()
        jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 16)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            results = list(ex.map(lambda s: _compile(s, flags, verbose), srcs))
        objs = [o for o, _ in results]
        manifest = "\n".join(os.path.basename(o) for o in objs) + "\n"
        out = target_path()
        try:
            with open(_manifest_path()) as f:
                linked = f.read()
        except OSError:
            linked = None
        if force or linked != manifest or not os.path.exists(out):
            tmp = f"{out}.{os.getpid()}.tmp"
            cmd = (
                [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp]
                + objs
                + [f"-L{ROCM}/lib", "-lrccl", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]
            )
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
            os.replace(tmp, out)
            with open(_manifest_path(), "w") as f:
                f.write(manifest)
        elif is_stale():  # same objects, but a source was touched after the link: refresh the stamp
            os.utime(out, None)
    return out


def build_sanitized(out_dir: str, verbose: bool = False) -> str:
    """Host-ASan variant of the extension in ``out_dir`` (never the in-tree module): the host C++
    runtime (``*.cpp``: bindings, RCCL communicator / bucket reducer / peer exchange, step
    executor) is compiled with ``-Xarch_host -fsanitize=address`` and linked with the regular
    objects of the HIP sources (their device code cannot be sanitized on this pool anyway).
    Load it with the clang ASan runtime preloaded (``asan_runtime()``); tests/test_sanitize_cpu.py
    drives it."""
    os.makedirs(out_dir, exist_ok=True)
    plain, asan = _flags(), _flags(sanitize=True)
    objs = []
    for src in _sources():
        o, _ = _compile(src, asan if src.endswith(".cpp") else plain, verbose)
        objs.append(o)
    out = os.path.join(out_dir, MODULE + sysconfig.get_config_var("EXT_SUFFIX"))
    cmd = ([os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-fsanitize=address",
            "-shared-libsan", "-o", out] + objs + [f"-L{ROCM}/lib", "-lrccl", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"ASan link failed:\n{r.stdout}\n{r.stderr}")
    return out


def asan_runtime() -> str:
    """Path of the clang ASan runtime hipcc links against (LD_PRELOAD it into a plain python)."""
    r = subprocess.run([os.path.join(ROCM, "bin", "hipcc"), "-print-file-name=libclang_rt.asan-x86_64.so"],
                       capture_output=True, text=True)
    return r.stdout.strip()


def is_stale() -> bool:
    out = target_path()
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in _sources() + _headers())


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
