"""Builds the native pieces in-tree (no pip, no JIT cache; the .so files travel with
the repo snapshot to the GPU box):

* ``k8s_gpu_device_plugin_amd/_native*.so``   C++17 core (amdsmi backend, fixture
  backend, xGMI allocator, protobuf hot paths, exporter, epoll httpd, inotify,
  native HTTP/2 gRPC server) + pybind11 bindings, linked against ``libamd_smi``.
* ``k8s_gpu_device_plugin_amd/ops/libamdgpu_canary.so``  HIP/CDNA4 health canary,
  ``hipcc --offload-arch=gfx950``.
* ``k8s_gpu_device_plugin_amd/_native_bench*.so``  the load generators and latency
  probes of ``bench.py``, ``scripts/`` and the tests (``tests/native/loadgen.cpp``,
  ``tests/native/bench_bindings.cpp``) over the same core objects.  Harness only: the
  plugin never imports it, so no DaemonSet pod carries it.
* ``build/native_selftest[-asan|-tsan]``  standalone C++ self-test (``tests/native/
  selftest.cpp``, no Python) for sanitizer runs.
* ``build/fuzz/fuzz_<target>``  libFuzzer + ASan + UBSan binaries (amdclang++, sources in
  ``tests/native/fuzz/``) for every parser that faces a peer: ``pbwire`` (kubelet protobuf
  + allocator contract), ``hpack``, ``grpc`` (HTTP/2 server on its socket), ``http``
  (HTTP/1.1 ops server).

Usage: ``python -m k8s_gpu_device_plugin_amd._build [--force] [--sanitize address|thread]
[--fuzz TARGET... --fuzz-seconds N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures
import os
import platform
import shutil
import subprocess
import sys
import sysconfig
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
NATIVE_DIR = os.path.join(ROOT, "native")
HARNESS_DIR = os.path.join(ROOT, "tests", "native")  # C++ test / bench harness
BUILD_DIR = os.path.join(ROOT, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
OFFLOAD_ARCH = "gfx950"

CORE_SOURCES = [
    "common.cpp",
    "lanes.cpp",
    "backend.cpp",
    "fixture_backend.cpp",
    "amdsmi_backend.cpp",
    "drm_reset.cpp",
    "core_escape.cpp",
    "allocator.cpp",
    "device_table.cpp",
    "health.cpp",
    "telemetry.cpp",
    "httpd.cpp",
    "watch.cpp",
    "hpack.cpp",
    "grpc_h2.cpp",
    "profiler.cpp",
]
BINDING_SOURCES = ["bindings.cpp"]
BENCH_SOURCES = ["loadgen.cpp", "bench_bindings.cpp"]  # in HARNESS_DIR
FUZZ_TARGETS = ("pbwire", "hpack", "grpc", "http")
FUZZ_DIR = os.path.join(HARNESS_DIR, "fuzz")
CANARY_SOURCES = [os.path.join(PKG_DIR, "ops", f) for f in ("canary.hip", "datapath.hip")]
CANARY_HEADERS = [os.path.join(PKG_DIR, "ops", "canary_common.h")]
CANARY_LIB = os.path.join(PKG_DIR, "ops", "libamdgpu_canary.so")


def native_ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, "_native" + suffix)


def bench_ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, "_native_bench" + suffix)


def _headers():
    return [os.path.join(d, f) for d in (NATIVE_DIR, HARNESS_DIR) if os.path.isdir(d)
            for f in os.listdir(d) if f.endswith(".h")]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, what: str) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("%s failed (%d):\n%s\n%s" % (what, proc.returncode, " ".join(cmd), proc.stdout))


def _cxx() -> str:
    return os.environ.get("CXX", "g++")


def _common_flags(sanitize: str | None):
    flags = ["-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-pthread",
             "-I" + NATIVE_DIR, "-I" + os.path.join(ROCM, "include")]
    if sanitize:
        flags += ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=" + sanitize]
        if sanitize == "address":
            flags.append("-fsanitize=undefined")
    else:
        flags += ["-O2", "-g1"]
    if platform.machine() in ("x86_64", "AMD64"):
        # x86-64-v2 (POPCNT, SSE4.2): every EPYC host of an MI355X has it, and without it
        # each __builtin_popcount in the allocator's scoring is a libgcc call
        flags.append("-march=x86-64-v2")
    return flags


def _link_libs():
    return ["-L" + os.path.join(ROCM, "lib"), "-lamd_smi", "-Wl,-rpath," + os.path.join(ROCM, "lib"),
            "-lz", "-pthread"]


def _compile_objects(sources, obj_dir, extra_flags, force, jobs, cxx=None, src_dir=NATIVE_DIR):
    os.makedirs(obj_dir, exist_ok=True)
    hdrs = _headers()
    cxx = cxx or _cxx()
    # objects built with other flags (or another compiler) are stale too
    stamp = os.path.join(obj_dir, ".flags")
    want = " ".join([cxx] + list(extra_flags))
    try:
        with open(stamp) as f:
            force = force or f.read() != want
    except OSError:
        force = True
    todo, objs = [], []
    for s in sources:
        src = os.path.join(src_dir, s)
        obj = os.path.join(obj_dir, s.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            todo.append((src, obj))

    def one(pair):
        src, obj = pair
        started = time.time()
        _run([cxx] + extra_flags + ["-c", src, "-o", obj], "compile " + os.path.basename(src))
        # the object is as old as the sources it read: one edited while it compiled (a
        # header changed under a long ASan build) leaves it stale for the next build
        os.utime(obj, (started, started))

    if todo:
        with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(one, todo))
    with open(stamp, "w") as f:
        f.write(want)
    return objs, bool(todo)


def build_native(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    import pybind11

    jobs = jobs or min(8, os.cpu_count() or 4)
    out = native_ext_path()
    flags = _common_flags(None)
    core_objs, core_changed = _compile_objects(CORE_SOURCES, os.path.join(BUILD_DIR, "obj"), flags, force, jobs)
    py_flags = flags + ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
                        "-fvisibility=hidden"]
    bind_objs, bind_changed = _compile_objects(BINDING_SOURCES, os.path.join(BUILD_DIR, "obj_py"), py_flags,
                                               force, jobs)
    if force or core_changed or bind_changed or not os.path.exists(out):
        tmp = out + ".tmp"
        _run([_cxx(), "-shared", "-o", tmp] + bind_objs + core_objs + _link_libs(), "link _native")
        os.replace(tmp, out)
        if verbose:
            print("built", os.path.relpath(out, ROOT))
    return out


def build_bench(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    """The harness extension (``_native_bench``): load generators and latency probes,
    linked with the same core objects as ``_native``."""
    import pybind11

    jobs = jobs or min(8, os.cpu_count() or 4)
    out = bench_ext_path()
    flags = _common_flags(None) + ["-I" + HARNESS_DIR]
    core_objs, core_changed = _compile_objects(CORE_SOURCES, os.path.join(BUILD_DIR, "obj"), _common_flags(None),
                                               force, jobs)
    py_flags = flags + ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-fvisibility=hidden"]
    objs, changed = _compile_objects(BENCH_SOURCES, os.path.join(BUILD_DIR, "obj_bench"), py_flags, force, jobs,
                                     src_dir=HARNESS_DIR)
    # the core objects are shared with _native: build_native may have refreshed them first
    if force or core_changed or changed or _stale(out, core_objs + objs):
        tmp = out + ".tmp"
        _run([_cxx(), "-shared", "-o", tmp] + objs + core_objs + _link_libs(), "link _native_bench")
        os.replace(tmp, out)
        if verbose:
            print("built", os.path.relpath(out, ROOT))
    return out


def sanitized_ext_path(sanitize: str) -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(BUILD_DIR, "ext-" + sanitize, "_native" + suffix)


def build_native_sanitized(sanitize: str, force: bool = False) -> str:
    """The pybind11 extension itself instrumented (ASan+UBSan or TSan), loaded through
    ``AMDGPU_DP_NATIVE_SO`` by a Python that preloads the sanitizer runtime, so the
    integration tests (kubelet stub, manager, both servers) run against it."""
    flags = _common_flags(sanitize)
    jobs = min(8, os.cpu_count() or 4)
    core, c1 = _compile_objects(CORE_SOURCES, os.path.join(BUILD_DIR, "obj-" + sanitize), flags, force, jobs)
    import pybind11
    py_flags = flags + ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-fvisibility=hidden"]
    bind, c2 = _compile_objects(BINDING_SOURCES, os.path.join(BUILD_DIR, "obj_py-" + sanitize), py_flags, force, jobs)
    out = sanitized_ext_path(sanitize)
    if force or c1 or c2 or not os.path.exists(out):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        link = [_cxx(), "-shared", "-fsanitize=" + sanitize] + (["-fsanitize=undefined"] if sanitize == "address" else [])
        _run(link + ["-o", out] + bind + core + _link_libs(), "link sanitized _native")
    return out


def sanitizer_runtime(sanitize: str) -> str:
    """Path of the compiler's shared sanitizer runtime (to LD_PRELOAD into python)."""
    lib = {"address": "libasan.so", "thread": "libtsan.so"}[sanitize]
    out = subprocess.run([_cxx(), "-print-file-name=" + lib], stdout=subprocess.PIPE, text=True).stdout.strip()
    if not out or not os.path.isabs(out) or not os.path.exists(out):
        raise RuntimeError("%s not found by %s" % (lib, _cxx()))
    return os.path.realpath(out)


def build_selftest(sanitize: str | None = None, force: bool = False) -> str:
    """Standalone C++ self-test binary (optionally ASan+UBSan or TSan instrumented)."""
    tag = {"address": "-asan", "thread": "-tsan", None: ""}[sanitize]
    obj_dir = os.path.join(BUILD_DIR, "obj_selftest" + tag)
    flags = _common_flags(sanitize)
    objs, changed = _compile_objects(CORE_SOURCES, obj_dir, flags, force, min(8, os.cpu_count() or 4))
    st, st_changed = _compile_objects(["selftest.cpp"], obj_dir, flags, force, 1, src_dir=HARNESS_DIR)
    objs, changed = objs + st, changed or st_changed
    exe = os.path.join(BUILD_DIR, "native_selftest" + tag)
    if force or changed or not os.path.exists(exe):
        link = [_cxx()] + (["-fsanitize=" + sanitize] if sanitize else [])
        if sanitize == "address":
            link.append("-fsanitize=undefined")
        _run(link + ["-o", exe] + objs + _link_libs(), "link selftest")
    return exe


def clangxx_path() -> str:
    p = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")
    if not os.path.exists(p):
        raise RuntimeError("libFuzzer builds need ROCm's clang++ (%s)" % p)
    return p


def build_fuzzer(target: str, force: bool = False) -> str:
    """libFuzzer binary for one target, ASan + UBSan, coverage on the core sources too.

    ``-mllvm -asan-globals=0``: ROCm's clang + libstdc++ 11 trips ASan's global
    alignment/ODR check on merged string literals (a false positive); heap, stack and
    UB checks are unaffected."""
    if target not in FUZZ_TARGETS:
        raise ValueError("unknown fuzz target %r (have %s)" % (target, ", ".join(FUZZ_TARGETS)))
    cxx = clangxx_path()
    san = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-mllvm", "-asan-globals=0",
           "-fno-sanitize-recover=undefined"]
    base = [f for f in _common_flags(None) if f not in ("-O2", "-g1")] + san
    core, core_changed = _compile_objects(CORE_SOURCES, os.path.join(BUILD_DIR, "obj_fuzz"),
                                          base + ["-fsanitize=fuzzer-no-link"], force, min(8, os.cpu_count() or 4),
                                          cxx=cxx)
    harness, h_changed = _compile_objects(["fuzz_%s.cpp" % target], os.path.join(BUILD_DIR, "obj_fuzz"),
                                          base + ["-fsanitize=fuzzer-no-link", "-I" + FUZZ_DIR], force, 1,
                                          cxx=cxx, src_dir=FUZZ_DIR)
    exe = os.path.join(BUILD_DIR, "fuzz", "fuzz_" + target)
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    if force or core_changed or h_changed or not os.path.exists(exe):
        _run([cxx, "-fsanitize=fuzzer,address,undefined", "-o", exe] + harness + core + _link_libs(),
             "link fuzz_" + target)
    return exe


def run_fuzzer(target: str, seconds: float = 10.0, force: bool = False, extra_args=()) -> subprocess.CompletedProcess:
    """Builds ``target``, writes its seed corpus, fuzzes for ``seconds``.  Crashes /
    hangs are saved under ``build/fuzz/artifacts/`` and make the return code non-zero."""
    exe = build_fuzzer(target, force=force)
    corpus = os.path.join(BUILD_DIR, "fuzz", "corpus", target)
    artifacts = os.path.join(BUILD_DIR, "fuzz", "artifacts") + os.sep
    os.makedirs(corpus, exist_ok=True)
    os.makedirs(artifacts, exist_ok=True)
    seeded = subprocess.run([exe], env=dict(os.environ, FUZZ_WRITE_SEEDS=corpus), stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    if seeded.returncode != 0:
        raise RuntimeError("fuzz_%s: writing seeds failed:\n%s" % (target, seeded.stdout[-2000:]))
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    cmd = [exe, corpus, "-max_total_time=%d" % max(1, int(seconds)), "-timeout=10", "-rss_limit_mb=4096",
           "-max_len=8192", "-print_final_stats=1", "-artifact_prefix=" + artifacts + target + "-"] + list(extra_args)
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    with open(os.path.join(BUILD_DIR, "fuzz", "fuzz_%s.log" % target), "w") as f:
        f.write(p.stdout)
    return p


def hipcc_path() -> str | None:
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else shutil.which("hipcc")


def build_canary(force: bool = False, verbose: bool = True) -> str:
    """hipcc the CDNA4 health-canary kernel library for gfx950 only."""
    hipcc = hipcc_path()
    if hipcc is None:
        raise RuntimeError("hipcc not found under %s/bin" % ROCM)
    if force or _stale(CANARY_LIB, CANARY_SOURCES + CANARY_HEADERS):
        tmp = CANARY_LIB + ".tmp"
        _run([hipcc, "--offload-arch=" + OFFLOAD_ARCH, "-O3", "-std=c++17", "-shared", "-fPIC",
              "-Wall", "-o", tmp] + CANARY_SOURCES, "hipcc canary")
        os.replace(tmp, CANARY_LIB)
        if verbose:
            print("built", os.path.relpath(CANARY_LIB, ROOT))
    return CANARY_LIB


def build_all(force: bool = False) -> None:
    build_native(force=force)
    build_bench(force=force)
    build_canary(force=force)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread"], default=None,
                    help="build the native self-test with a sanitizer instead")
    ap.add_argument("--sanitize-ext", choices=["address", "thread"], default=None,
                    help="build the pybind11 extension with a sanitizer (under build/ext-<name>/)")
    ap.add_argument("--selftest", action="store_true", help="also build (and run) the native self-test")
    ap.add_argument("--no-canary", action="store_true")
    ap.add_argument("--fuzz", nargs="*", choices=FUZZ_TARGETS, default=None,
                    help="build and run libFuzzer targets (all when none named)")
    ap.add_argument("--fuzz-seconds", type=float, default=30.0)
    args = ap.parse_args(argv)
    if args.fuzz is not None:
        rc = 0
        for t in args.fuzz or FUZZ_TARGETS:
            p = run_fuzzer(t, args.fuzz_seconds, force=args.force)
            tail = [ln for ln in p.stdout.splitlines() if ln.startswith(("#", "Done", "stat::", "=="))][-4:]
            print("fuzz_%s: rc=%d\n  %s" % (t, p.returncode, "\n  ".join(tail)))
            rc = rc or p.returncode
        return rc
    if args.sanitize_ext:
        print("built", os.path.relpath(build_native_sanitized(args.sanitize_ext, force=args.force), ROOT))
        print("run with: LD_PRELOAD=%s AMDGPU_DP_NATIVE_SO=<that path>" % sanitizer_runtime(args.sanitize_ext))
        return 0
    if args.sanitize or args.selftest:
        exe = build_selftest(args.sanitize, force=args.force)
        print("built", os.path.relpath(exe, ROOT))
        r = subprocess.run([exe])
        return r.returncode
    build_native(force=args.force)
    build_bench(force=args.force)
    if not args.no_canary:
        build_canary(force=args.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
