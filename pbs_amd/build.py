"""In-tree native build for gpbs (no JIT cache, no pip install).

Produces, under ``pbs_amd/lib/``:

* ``libgpbs.so``      host C++17 scheduler core + C ABI (csrc/core, obs, ipc,
                      counters, actuate, api).  Built with g++.
* ``libgpbs_hip.so``  gfx950 HIP kernels + the GPU runtime (partition table,
                      software counters, tenant runners).  Built with hipcc
                      ``--offload-arch=gfx950`` and linked against libgpbs.so.

Both are rebuilt only when a source is newer than the library.  ``python -m
pbs_amd.build`` builds everything; ``__graft_entry__.build()`` calls this.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "pbs_amd", "lib")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

CORE_DIRS = ["core", "obs", "ipc", "counters", "actuate", "api", "comm"]
HIP_DIR = "hip"


def _srcs(dirs, exts):
    out = []
    for d in dirs:
        for e in exts:
            out += sorted(glob.glob(os.path.join(CSRC, d, "*" + e)))
    return out


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _digest(deps, extra=""):
    """Content hash of the dependencies, keyed by their path RELATIVE to the
    repo: the same tree hashes the same wherever it is checked out (the GPU
    box runs a copy under another root and must not rebuild)."""
    import hashlib
    h = hashlib.sha1(extra.encode())
    for d in sorted(deps, key=lambda x: os.path.relpath(x, ROOT)):
        h.update(os.path.relpath(d, ROOT).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


class _BuildLock:
    """Inter-process lock around a build (torchrun ranks and test
    subprocesses load the libraries at the same time; two concurrent builds
    sharing one object directory could link a half-written object)."""

    def __enter__(self):
        import fcntl
        os.makedirs(LIBDIR, exist_ok=True)
        self.f = open(os.path.join(LIBDIR, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        import fcntl
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def _lib_stale(target, deps, extra=""):
    """A library is stale when its stamp (content hash of every dependency
    and the flags) differs -- robust to copies that do not keep mtimes (the
    GPU-box snapshot), unlike an mtime comparison."""
    stamp = target + ".stamp"
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(deps, extra)


def _link_atomic(cmd_prefix, target, cmd_suffix, verbose, deps, extra=""):
    """Link into a temp file and rename over the target: a process that has
    the old library mapped keeps it, a concurrent loader never sees a torn
    file."""
    tmp = f"{target}.tmp.{os.getpid()}"
    _run(cmd_prefix + ["-o", tmp] + cmd_suffix, verbose)
    os.replace(tmp, target)
    with open(target + ".stamp", "w") as f:
        f.write(_digest(deps, extra))


def _run(cmd, verbose):
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("native build failed: " + " ".join(cmd[:3]) + " ...")
    return r.stdout


def _compile_parallel(jobs, verbose):
    """jobs: list of (cmd, obj). Runs up to 8 at a time."""
    procs = []
    maxp = int(os.environ.get("GPBS_BUILD_JOBS", "8"))
    pending = list(jobs)
    errors = []
    while pending or procs:
        while pending and len(procs) < maxp:
            cmd, obj = pending.pop(0)
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True), cmd))
        p, cmd = procs.pop(0)
        out, _ = p.communicate()
        if p.returncode != 0:
            errors.append(out)
    if errors:
        sys.stderr.write("\n".join(errors))
        raise RuntimeError("native build failed")


def build_core(verbose=False, sanitize: str | None = None):
    """Build libgpbs.so.  sanitize in {None, 'address', 'thread', 'undefined'}."""
    with _BuildLock():
        return _build_core(verbose, sanitize)


def _build_core(verbose=False, sanitize: str | None = None):
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = _srcs(CORE_DIRS, [".cpp"])
    name = "libgpbs.so" if not sanitize else f"libgpbs_{sanitize}.so"
    target = os.path.join(LIBDIR, name)
    deps = srcs + _headers() + [__file__]
    if not _lib_stale(target, deps, str(sanitize)):
        return target
    objdir = os.path.join(ROOT, "build", "core" + (("_" + sanitize) if sanitize else ""))
    os.makedirs(objdir, exist_ok=True)
    flags = ["-std=c++17", "-O2", "-g", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread",
             "-I" + os.path.join(CSRC, "include"), "-fvisibility=default"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-O1"]
    jobs = []
    objs = []
    for s in srcs:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        obj = os.path.join(objdir, rel + ".o")
        objs.append(obj)
        if _stale(obj, [s] + _headers()):
            jobs.append((["g++"] + flags + ["-c", s, "-o", obj], obj))
    _compile_parallel(jobs, verbose)
    suffix = objs + ["-pthread", "-lrt"] + ([f"-fsanitize={sanitize}"] if sanitize else [])
    _link_atomic(["g++", "-shared"], target, suffix, verbose, deps, str(sanitize))
    return target


def hipcc():
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build_hip(verbose=False):
    """Build libgpbs_hip.so for gfx950 (cross-compiles without a GPU)."""
    core = build_core(verbose)
    with _BuildLock():
        return _build_hip(verbose)


def _build_hip(verbose=False):
    srcs = _srcs([HIP_DIR], [".hip", ".cpp"])
    if not srcs:
        return None
    target = os.path.join(LIBDIR, "libgpbs_hip.so")
    hdrs = _headers() + sorted(glob.glob(os.path.join(CSRC, HIP_DIR, "*.hpp")))
    deps = srcs + hdrs + [__file__] + _srcs(CORE_DIRS, [".cpp"]) + _headers()
    if not _lib_stale(target, deps, ARCH):
        return target
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    flags = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-I" + os.path.join(CSRC, "include"),
             "-Wno-unused-result", "-munsafe-fp-atomics"]
    jobs, objs = [], []
    for s in srcs:
        obj = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(obj)
        if _stale(obj, [s] + hdrs + [__file__]):
            lang = ["-x", "hip"] if s.endswith(".hip") or s.endswith(".cpp") else []
            jobs.append(([hipcc()] + flags + lang + ["-c", s, "-o", obj], obj))
    _compile_parallel(jobs, verbose)
    _link_atomic([hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}"], target,
                 objs + ["-L" + LIBDIR, "-lgpbs", "-Wl,-rpath,$ORIGIN", "-L/opt/rocm/lib", "-lrocprofiler-sdk", "-lrocprofiler-sdk-roctx", "-lhsa-runtime64",
                         "-Wl,-rpath,/opt/rocm/lib", "-pthread"], verbose, deps, ARCH)
    return target


def build_all(verbose=False):
    core = build_core(verbose)
    hip = build_hip(verbose)
    return core, hip


if __name__ == "__main__":
    v = "-v" in sys.argv
    san = None
    for a in sys.argv[1:]:
        if a.startswith("--sanitize="):
            san = a.split("=", 1)[1]
    if san:
        print(build_core(v, sanitize=san))
    else:
        print(build_all(v))
