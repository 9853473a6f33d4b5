"""In-tree native build: HIP kernels (gfx950) + C++ runtime / networking.

Everything is compiled with the ROCm toolchain directly (hipcc / g++), no
torch.utils.cpp_extension and no hipify step.  Artefacts land inside the
package (``p2p_llm_chat_go_amd/_lib``) so that they travel with the repo
snapshot to the GPU box.  Targets are rebuilt only when a source or header is
newer than the artefact.

Usage:  python -m p2p_llm_chat_go_amd._build [--force] [--jobs N] [--only kernels|net|...]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "p2p_llm_chat_go_amd")
LIBDIR = os.path.join(PKG, "_lib")
BINDIR = os.path.join(ROOT, "bin")
BUILDDIR = os.path.join(ROOT, "build")
CSRC = os.path.join(ROOT, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("P2P_GPU_ARCH", "gfx950")

HIPCC = os.path.join(ROCM, "bin", "hipcc")
CXX = os.environ.get("CXX", "g++")

KERNEL_LIB = os.path.join(LIBDIR, "libp2p_kernels.so")


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _stale(target, deps):
    return (not os.path.exists(target)) or os.path.getmtime(target) < _newest(deps)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n  %s\n%s" % (" ".join(cmd), r.stdout[-8000:]))
    return r.stdout


def sources_digest(paths) -> str:
    """sha256 over the (relative path, bytes) of every source and header a library is built
    from: recorded next to the library at link time (``<lib>.stamp``) and compared by the
    loader (ops/_lib.py), so a binary that no build of the current sources produced is
    refused instead of silently tested (What's weak #8)."""
    import hashlib

    h = hashlib.sha256()
    for p in sorted(set(paths)):
        h.update(os.path.relpath(p, ROOT).encode())
        h.update(b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def kernel_sources(experimental=False):
    """(sources, headers) of the kernel library (or of the experimental one)."""
    kdir = os.path.join(CSRC, "kernels")
    sub = "experimental" if experimental else "kernels"
    srcs = sorted(glob.glob(os.path.join(CSRC, sub, "*.hip")))
    hdrs = _headers(kdir)
    if experimental:  # probe builds #include kernel sources (wide_stamp.hip: wide_gemm.hip)
        hdrs += sorted(glob.glob(os.path.join(kdir, "*.hip")))
    return srcs, hdrs


def _write_stamp(out_lib, srcs, hdrs):
    import json

    with open(out_lib + ".stamp", "w") as f:
        json.dump({"sources_sha256": sources_digest(list(srcs) + list(hdrs)),
                   "n_files": len(set(srcs) | set(hdrs)), "arch": ARCH}, f)


def _headers(d):
    return glob.glob(os.path.join(d, "*.h")) + glob.glob(os.path.join(CSRC, "include", "*.h"))


EXPERIMENTAL_LIB = os.path.join(LIBDIR, "libp2p_experimental.so")


# Kernels whose k loop streams through inline-asm loads (csrc/kernels/wide_gemm.hip): the
# compiler does not know those registers are still in flight, so a spill of one would read
# it before it lands.  Their translation units must compile with zero scratch.
NO_SCRATCH = {"wide_gemm.hip", "tiled_gemm.hip"}


def check_no_scratch(src, remarks: str, obj=None):
    """Raise if any kernel of ``src`` uses scratch (the -Rpass-analysis=kernel-resource-usage
    remarks of its compile)."""
    import re

    bad, name = [], None
    for line in remarks.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and int(m.group(1)) > 0:
            bad.append("%s (%s B/lane)" % (name, m.group(1)))
    if bad:
        if obj and os.path.exists(obj):
            os.remove(obj)
        raise RuntimeError("%s: kernels with scratch (asm-pipelined loads must not spill): %s"
                           % (os.path.basename(src), "; ".join(bad)))


def build_kernels(force=False, jobs=8, experimental=False):
    """Compile csrc/kernels/*.hip for gfx950 into one shared library (C ABI, ctypes).

    experimental=True builds csrc/experimental/*.hip (measured-negative fusions and
    hardware probes kept for the record and their benches) into a separate
    ``libp2p_experimental.so`` instead; no default engine path loads it."""
    kdir = os.path.join(CSRC, "kernels")
    srcs, hdrs = kernel_sources(experimental)
    odir = os.path.join(BUILDDIR, "experimental" if experimental else "kernels")
    out_lib = EXPERIMENTAL_LIB if experimental else KERNEL_LIB
    os.makedirs(odir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    flags = [
        "--offload-arch=%s" % ARCH, "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
        "-Wno-unused-result", "-I", os.path.join(CSRC, "include"), "-I", kdir,
    ]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(odir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append((s, o))
    def compile_one(s, o):
        if os.path.basename(s) not in NO_SCRATCH:
            return _run([HIPCC] + flags + ["-c", s, "-o", o])
        out = _run([HIPCC] + flags + ["-Rpass-analysis=kernel-resource-usage", "-c", s, "-o", o])
        check_no_scratch(s, out, o)
        return out

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(compile_one, s, o) for s, o in todo]
        for f in futs:
            f.result()
    # a source removed from the directory leaves its object behind: relink from the
    # current source list whenever the library holds objects it should not
    listed = out_lib + ".objs"
    prev = open(listed).read().split("\n") if os.path.exists(listed) else None
    if prev != objs and os.path.exists(out_lib):
        os.remove(out_lib)
    if force or todo or _stale(out_lib, objs):
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=%s" % ARCH] + objs + ["-o", out_lib])
        with open(listed, "w") as f:
            f.write("\n".join(objs))
    _write_stamp(out_lib, srcs, hdrs)
    return out_lib


def _py_ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def build_native(force=False, jobs=8):
    """C++ runtime + networking: static objects, pybind11 module, and daemons."""
    import pybind11  # noqa: F401  (build dependency, present in the image)

    subdirs = ["net", "runtime"]
    odir = os.path.join(BUILDDIR, "native")
    os.makedirs(odir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    inc = ["-I", os.path.join(CSRC, "include"), "-I", CSRC]
    base = ["-O2", "-g", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-pthread"] + inc
    srcs = []
    for d in subdirs:
        srcs += sorted(glob.glob(os.path.join(CSRC, d, "*.cc")))
    hdrs = []
    for d in subdirs + ["include"]:
        hdrs += glob.glob(os.path.join(CSRC, d, "*.h"))
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(odir, os.path.relpath(s, CSRC).replace(os.sep, "_") + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, [CXX] + base + ["-c", s, "-o", o]) for s, o in todo]:
            f.result()
    if not objs:
        return []
    libs = ["-lssl", "-lcrypto", "-pthread"]
    outs = []
    # static archive for the daemons
    ar = os.path.join(odir, "libp2pnative.a")
    if force or todo or _stale(ar, objs):
        if os.path.exists(ar):
            os.remove(ar)
        _run(["ar", "rcs", ar] + objs)
    # daemons
    for app in sorted(glob.glob(os.path.join(CSRC, "apps", "*.cc"))):
        name = os.path.splitext(os.path.basename(app))[0]
        exe = os.path.join(BINDIR, name)
        if force or _stale(exe, [app, ar] + hdrs):
            _run([CXX] + base + [app, ar, "-o", exe] + libs + ["-ldl"])
        outs.append(exe)
    # pybind11 module
    import pybind11

    bind = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cc")))
    if bind:
        mod = os.path.join(LIBDIR, "_native" + _py_ext_suffix())
        pyinc = sysconfig.get_paths()["include"]
        if force or _stale(mod, bind + [ar] + hdrs):
            _run([CXX] + base + ["-shared", "-I", pybind11.get_include(), "-I", pyinc] + bind
                 + [ar, "-o", mod] + libs + ["-ldl"])
        outs.append(mod)
    # engine C ABI (embeds the interpreter that drives the Python/HIP engine)
    eng_src = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cc")))
    if eng_src:
        lib = os.path.join(LIBDIR, "libp2p_engine.so")
        pyinc = sysconfig.get_paths()["include"]
        pylib = ["-L" + (sysconfig.get_config_var("LIBDIR") or "/usr/lib"),
                 "-lpython%s" % sysconfig.get_config_var("VERSION")]
        ehdrs = glob.glob(os.path.join(CSRC, "engine", "*.h"))
        # (links the runtime archive for the JSON codec; the loop itself is driven through
        # the table of the pybind module that owns it, runtime/loop_capi.h)
        if force or _stale(lib, eng_src + ehdrs + hdrs + [ar]):
            _run([CXX] + base + ["-shared", "-I", pyinc] + eng_src + [ar, "-o", lib] + pylib
                 + libs + ["-ldl"])
        outs.append(lib)
    return outs


SANITIZERS = {
    # SURVEY.md §5 "Race detection / sanitizers": CPU-side variants of the daemons
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


# ROCm's clang: its compiler-rt TSan intercepts pthread_cond_clockwait (used by
# libstdc++'s condition_variable::wait_for); GCC 11's libtsan does not, which
# makes every timed wait look like a double lock / race.
SAN_CXX = os.environ.get("P2P_SAN_CXX", os.path.join(ROCM, "lib", "llvm", "bin", "clang++"))


def build_sanitized(kind: str, force=False, jobs=8):
    """Daemons (directory / node / relay) built with ASan+UBSan or TSan into bin/<kind>/."""
    san = SANITIZERS[kind]
    cxx = SAN_CXX if os.path.exists(SAN_CXX) else CXX
    subdirs = ["net", "runtime"]
    odir = os.path.join(BUILDDIR, "native-" + kind)
    bdir = os.path.join(BINDIR, kind)
    os.makedirs(odir, exist_ok=True)
    os.makedirs(bdir, exist_ok=True)
    inc = ["-I", os.path.join(CSRC, "include"), "-I", CSRC]
    base = ["-O1", "-g", "-std=c++17", "-pthread"] + san + inc
    srcs, hdrs = [], []
    for d in subdirs:
        srcs += sorted(glob.glob(os.path.join(CSRC, d, "*.cc")))
    for d in subdirs + ["include"]:
        hdrs += glob.glob(os.path.join(CSRC, d, "*.h"))
    objs, todo = [], []
    for s_ in srcs:
        o = os.path.join(odir, os.path.relpath(s_, CSRC).replace(os.sep, "_") + ".o")
        objs.append(o)
        if force or _stale(o, [s_] + hdrs):
            todo.append((s_, o))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, [cxx] + base + ["-c", a, "-o", b]) for a, b in todo]:
            f.result()
    outs = []
    for app in sorted(glob.glob(os.path.join(CSRC, "apps", "*.cc"))):
        name = os.path.splitext(os.path.basename(app))[0]
        exe = os.path.join(bdir, name)
        if force or _stale(exe, [app] + objs + hdrs):
            _run([cxx] + base + [app] + objs + ["-o", exe, "-lssl", "-lcrypto", "-pthread", "-ldl"])
        outs.append(exe)
    return outs


def build(force=False, jobs=8, only=None, experimental=None):
    outs = []
    if experimental is None:
        # on by default: the experimental library's tests run on the GPU box, so the binary
        # they load must be built from HEAD like the rest (P2P_BUILD_EXPERIMENTAL=0 skips it)
        experimental = os.environ.get("P2P_BUILD_EXPERIMENTAL", "1") == "1"
    if only in (None, "kernels", "experimental"):
        if shutil.which(HIPCC) or os.path.exists(HIPCC):
            if only != "experimental":
                outs.append(build_kernels(force, jobs))
            if experimental or only == "experimental":
                outs.append(build_kernels(force, jobs, experimental=True))
        else:
            print("hipcc not found; skipping HIP kernels", file=sys.stderr)
    if only in (None, "native"):
        outs += build_native(force, jobs)
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", choices=["kernels", "native", "experimental"], default=None)
    ap.add_argument("--sanitize", choices=sorted(SANITIZERS), default=None,
                    help="build only the sanitizer variant of the daemons into bin/<kind>/")
    a = ap.parse_args(argv)
    if a.sanitize:
        for o in build_sanitized(a.sanitize, a.force, a.jobs):
            print(o)
        return
    for o in build(a.force, a.jobs, a.only):
        print(o)


if __name__ == "__main__":
    main()
