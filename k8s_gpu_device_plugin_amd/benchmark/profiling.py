"""``benchmark: true`` profiling harness.

Reference ``benchmark/benchmark.go``: creates ``./temp_bench*``, starts a CPU pprof,
sets heap/block/mutex sampling rates (``:54-89``) and on ``Stop`` writes
``cpu.prof``/``mem.prof``/``block.prof``/``mutex.prof`` (``:92-124``).  The Python
analogue writes ``cpu.prof`` (cProfile/pstats), ``mem.prof`` (tracemalloc top
allocations), ``threads.prof`` (stacks of every thread; the block/mutex analogue) and
``latency.prom`` (the native RPC/HTTP latency histograms, which is what the north-star
metrics need) and ``native.prof`` (a whole-process SIGPROF sample of every thread,
native code included - the true pprof analogue, since cProfile sees one Python thread;
``native/profiler.cpp``).  ``stop()`` is registered with ``atexit`` so it also runs on error exits
(defect D19).
"""
from __future__ import annotations

import atexit
import cProfile
import os
import pstats
import sys
import tempfile
import threading
import traceback
import tracemalloc

from ..utils.log import get_logger

log = get_logger("benchmark")


class Benchmark:
    def __init__(self, directory: str = "", render_metrics=None) -> None:
        if directory:
            os.makedirs(directory, exist_ok=True)
            self.dir = directory
        else:
            self.dir = tempfile.mkdtemp(prefix="temp_bench", dir=".")
        self.render_metrics = render_metrics
        self._prof: cProfile.Profile | None = None
        self._native = False
        self._stopped = False

    def run(self) -> None:
        tracemalloc.start(16)
        self._prof = cProfile.Profile()
        self._prof.enable()
        from .. import native
        self._native = native.load().prof_start(997)  # every thread, native code included
        atexit.register(self.stop)
        log.info("profiling to %s", self.dir)

    def stop(self) -> None:
        if self._stopped:
            return
        self._stopped = True
        if self._prof is not None:
            self._prof.disable()
            self._prof.dump_stats(os.path.join(self.dir, "cpu.prof"))
            with open(os.path.join(self.dir, "cpu.txt"), "w") as f:
                pstats.Stats(self._prof, stream=f).sort_stats("cumulative").print_stats(60)
        if self._native:
            from .. import native
            n = native.load()
            n.prof_stop()
            write_native_profile(os.path.join(self.dir, "native.prof"), symbolize(n.prof_histogram()),
                                 n.prof_dropped())
        if tracemalloc.is_tracing():
            snap = tracemalloc.take_snapshot()
            with open(os.path.join(self.dir, "mem.prof"), "w") as f:
                for stat in snap.statistics("lineno")[:100]:
                    f.write(str(stat) + "\n")
            tracemalloc.stop()
        with open(os.path.join(self.dir, "threads.prof"), "w") as f:
            frames = sys._current_frames()
            for t in threading.enumerate():
                f.write("--- thread %s (%s)\n" % (t.name, t.ident))
                if t.ident in frames:
                    f.write("".join(traceback.format_stack(frames[t.ident])))
        if self.render_metrics is not None:
            try:
                with open(os.path.join(self.dir, "latency.prom"), "w") as f:
                    f.write(self.render_metrics())
            except Exception as e:  # pragma: no cover
                log.error("latency dump failed: %s", e)
        log.info("profiles written to %s", self.dir)


def symbolize(rows, symbolizer: str | None = None) -> list:
    """(module, offset, dladdr symbol, samples) -> [(function, module, samples)], one row
    per function.  llvm-symbolizer (ROCm ships one) resolves internal functions from the
    -g line tables; without it, dladdr's nearest exported symbol is used."""
    import collections
    import shutil
    import subprocess
    exe = symbolizer or os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin",
                                     "llvm-symbolizer")
    if not os.path.exists(exe):
        exe = shutil.which("llvm-symbolizer") or ""
    names = {}
    keyed = [(m, off) for m, off, _, _ in rows if m != "?"]
    if exe and keyed:
        try:
            inp = "".join("%s 0x%x\n" % (m, off) for m, off in keyed)
            p = subprocess.run([exe, "--functions=linkage", "--demangle", "--no-inlines"], input=inp,
                               stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=120)
            blocks = [b.splitlines() for b in p.stdout.strip("\n").split("\n\n")]
            for key, blk in zip(keyed, blocks):
                if blk and blk[0] not in ("??", ""):
                    names[key] = blk[0]
        except (OSError, subprocess.SubprocessError):
            names = {}
    agg = collections.Counter()
    for m, off, sym, n in rows:
        fn = names.get((m, off)) or sym or "0x%x" % off
        agg[(fn, os.path.basename(m))] += n
    return [(fn, mod, n) for (fn, mod), n in agg.most_common()]


def write_native_profile(path: str, rows: list, dropped: int = 0, top: int = 80) -> None:
    total = sum(n for _, _, n in rows) or 1
    with open(path, "w") as f:
        f.write("# whole-process CPU samples (SIGPROF on CLOCK_PROCESS_CPUTIME_ID, overrun-weighted); %d samples, %d dropped\n"
                % (total, dropped))
        f.write("%8s %7s  %-40s %s\n" % ("samples", "share", "module", "function"))
        for fn, mod, n in rows[:top]:
            f.write("%8d %6.2f%%  %-40s %s\n" % (n, 100.0 * n / total, mod, fn))
