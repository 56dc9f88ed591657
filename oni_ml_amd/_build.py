"""Native build driver: compiles the CDNA4 HIP kernels and the C++ host runtime in-tree.

No torch.utils.cpp_extension / hipify is involved: HIP sources are compiled with
``hipcc --offload-arch=gfx950`` and linked with pybind11 bindings into
``oni_ml_amd/_lib/_onihip*.so``; the C++ host runtime (CSV parser, formatters,
lda-c reference EM, DNS parser) is compiled with ``g++`` into
``oni_ml_amd/_lib/_oninative*.so`` plus the standalone ``lda`` executable that
mirrors oni-lda-c's command line (reference call site ``ml_ops.sh:80``).

Builds are incremental: every artefact carries a stamp holding the hash of its
inputs (sources, headers, flags, compiler); an unchanged hash skips the step.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
import threading
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIB = Path(__file__).resolve().parent / "_lib"
OBJ = ROOT / "build" / "obj"

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = os.environ.get("ONI_OFFLOAD_ARCH", "gfx950")

_lock = threading.Lock()
# what the last build_all() did, per artefact: {"artefact", "action": compiled | up-to-date, "seconds"}
RECORD: list = []


def _note(out: Path, compiled: bool, t0: float):
    import time
    RECORD.append(dict(artefact=str(Path(out).relative_to(ROOT)), action="compiled" if compiled else "up-to-date",
                       seconds=round(time.perf_counter() - t0, 3)))


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_inc() -> str:
    import pybind11

    return pybind11.get_include()


def _py_inc() -> str:
    return sysconfig.get_paths()["include"]


def _hash(files, flags) -> str:
    h = hashlib.sha256()
    for f in sorted(str(x) for x in files):
        h.update(f.encode())
        h.update(Path(f).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _stale(out: Path, digest: str) -> bool:
    stamp = out.with_name(out.name + ".stamp")
    if not out.exists() or not stamp.exists():
        return True
    return stamp.read_text().strip() != digest


def _stamp(out: Path, digest: str):
    out.with_name(out.name + ".stamp").write_text(digest)


def _compile(src: Path, out: Path, cmd_prefix, flags, deps, verbose):
    import time
    t0 = time.perf_counter()
    digest = _hash([src] + list(deps), cmd_prefix + flags)
    if not _stale(out, digest):
        _note(out, False, t0)
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    _run(cmd_prefix + flags + ["-c", str(src), "-o", str(out)], verbose)
    _stamp(out, digest)
    _note(out, True, t0)
    return out


def _link(out: Path, objs, cmd, verbose):
    import time
    t0 = time.perf_counter()
    digest = _hash(objs, cmd)
    stale = _stale(out, digest)
    if stale:
        out.parent.mkdir(parents=True, exist_ok=True)
        # link to a temporary name, then rename: a reader (a running import, a tree snapshot) sees the
        # old library or the new one, never a half-written file
        tmp = out.with_name(out.name + ".tmp")
        cmd = list(cmd)
        i = cmd.index("-o")
        cmd[i + 1] = str(tmp)
        _run(cmd, verbose)
        os.replace(tmp, out)
        _stamp(out, digest)
    _note(out, stale, t0)


def hip_flags():
    return [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__", "-Wno-unused-result",
        "-munsafe-fp-atomics",
        f"-I{CSRC / 'hip'}",
    ]


def native_flags():
    # x86-64-v3 (AVX2, FMA: every EPYC host of an MI355X): the formatters' exact products take one
    # fused multiply-add; -ffp-contract=off keeps every other expression exactly as written
    return ["-O3", "-std=c++17", "-fPIC", "-march=x86-64-v3", "-ffp-contract=off", "-pthread",
            "-Wall", "-Wno-unused-function", "-Wno-sign-compare", f"-I{CSRC / 'native'}"]


def build_hip(verbose=False, jobs=8) -> Path:
    """Compile csrc/hip/*.hip (device kernels, gfx950) + bind_hip.cpp into _onihip."""
    out = LIB / ("_onihip" + _ext_suffix())
    hdrs = sorted((CSRC / "hip").glob("*.h"))
    srcs = sorted((CSRC / "hip").glob("*.hip"))
    bind = CSRC / "hip" / "bind_hip.cpp"
    flags = hip_flags()
    objs = []

    def one(src):
        o = OBJ / "hip" / (src.stem + ".o")
        extra = [f"-I{_pybind_inc()}", f"-I{_py_inc()}"] if src == bind else []
        return _compile(src, o, [HIPCC], flags + extra, hdrs, verbose)

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(one, srcs + [bind]))
    link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", str(out)] + [str(o) for o in objs]
    _link(out, objs, link, verbose)
    return out


def build_hip_exp(verbose=False, jobs=8) -> Path:
    """csrc/hip/experimental/ (E-step variants measured not faster, for their tests and benchmarks)
    into _onihip_exp: a module of its own, so the production code object and ml_ops never carry them."""
    out = LIB / ("_onihip_exp" + _ext_suffix())
    exp = CSRC / "hip" / "experimental"
    hdrs = sorted((CSRC / "hip").glob("*.h")) + sorted(exp.glob("*.h"))
    srcs = sorted(exp.glob("*.hip"))
    bind = exp / "bind_exp.cpp"
    flags = hip_flags()

    def one(src):
        o = OBJ / "hip_exp" / (src.stem + ".o")
        extra = [f"-I{_pybind_inc()}", f"-I{_py_inc()}"] if src == bind else []
        return _compile(src, o, [HIPCC], flags + extra, hdrs, verbose)

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(one, srcs + [bind]))
    link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", str(out)] + [str(o) for o in objs]
    _link(out, objs, link, verbose)
    return out


def build_native(verbose=False, jobs=8) -> Path:
    """Compile csrc/native/*.cpp (host runtime) into _oninative + the `lda` CLI binary."""
    cxx = os.environ.get("CXX", "g++")
    out = LIB / ("_oninative" + _ext_suffix())
    hdrs = sorted((CSRC / "native").glob("*.h"))
    srcs = [s for s in sorted((CSRC / "native").glob("*.cpp")) if s.name not in ("lda_main.cpp", "selftest.cpp")]
    bind = CSRC / "native" / "bind_native.cpp"
    if not bind.exists():
        return None
    lib_srcs = [s for s in srcs if s != bind]
    flags = native_flags()

    def one(src):
        o = OBJ / "native" / (src.stem + ".o")
        extra = [f"-I{_pybind_inc()}", f"-I{_py_inc()}"] if src == bind else []
        return _compile(src, o, [cxx], flags + extra, hdrs, verbose)

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(one, lib_srcs + [bind]))
    link = [cxx, "-shared", "-fPIC", "-pthread", "-o", str(out)] + [str(o) for o in objs]
    _link(out, objs, link, verbose)
    # standalone lda-c compatible executable
    main = CSRC / "native" / "lda_main.cpp"
    if main.exists():
        mo = one(main)
        exe = LIB / "lda"
        lib_objs = [o for o in objs if o.stem != "bind_native"]
        cmd = [cxx, "-pthread", "-o", str(exe), str(mo)] + [str(o) for o in lib_objs]
        _link(exe, [mo] + lib_objs, cmd, verbose)
    return out


def build_sanitized(kind: str = "thread", verbose=False) -> Path:
    """Native self-test executable under a host sanitizer (thread | address).

    GPU sanitizers are not available on this pool, so race / memory checking
    covers the multithreaded C++ runtime; the HIP kernels get
    their checks from host-side shape/index validation before every launch."""
    cxx = os.environ.get("CXX", "g++")
    san = {"thread": ["-fsanitize=thread"], "address": ["-fsanitize=address,undefined"]}[kind]
    outdir = ROOT / "build" / f"san_{kind}"
    outdir.mkdir(parents=True, exist_ok=True)
    srcs = [CSRC / "native" / f for f in ("table.cpp", "dns.cpp", "lda_ref.cpp", "selftest.cpp")]
    exe = outdir / "native_selftest"
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-march=x86-64-v3", "-pthread", f"-I{CSRC / 'native'}"] + san
    digest = _hash(srcs + sorted((CSRC / "native").glob("*.h")), flags)
    if _stale(exe, digest):
        _run([cxx] + flags + [str(s) for s in srcs] + ["-o", str(exe)], verbose)
        _stamp(exe, digest)
    return exe


def build_all(verbose=False, hip=True, native=True, experimental=False):
    """experimental: also build csrc/hip/experimental/ (only on request: ``python -m oni_ml_amd._build exp``;
    ml_ops never loads it, and its tests skip without it)."""
    with _lock:
        RECORD.clear()
        outs = []
        if native:
            o = build_native(verbose)
            if o is not None:
                outs.append(o)
        if hip:
            if not Path(HIPCC).exists():
                raise RuntimeError(f"hipcc not found at {HIPCC}")
            outs.append(build_hip(verbose))
            if experimental:
                outs.append(build_hip_exp(verbose))
            else:
                # a stale experimental module would travel with the tree and be mapped by its tests
                for p in LIB.glob("_onihip_exp*"):
                    p.unlink()
        return outs


def clean():
    shutil.rmtree(ROOT / "build", ignore_errors=True)
    for p in LIB.glob("*"):
        if p.name != "__init__.py":
            p.unlink()


if __name__ == "__main__":
    v = "-v" in sys.argv
    if "clean" in sys.argv:
        clean()
    print(build_all(verbose=v, experimental="exp" in sys.argv))
