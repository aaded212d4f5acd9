#!/usr/bin/env python3
"""Headline benchmark: device-resident GB/s of the 20-client wide_resnet16_8
parameter reduction (BASELINE.json metric, configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step is one aggregation of 20 client state_dicts (wide_resnet16_8,
CIFAR-10 layout: 82 fp32 keys + 16 int64 keys, B = 43,888,744 bytes) into the
global state — the reference's ``server_aggregate`` arithmetic
(train_fedavg.py:143-147) — with every input already resident in HBM.
``value`` = algorithmic bytes (N·B read + B written, SURVEY.md §8 d) / time.

N>1 (launched by torch.distributed.run, one rank per GPU): weak scaling,
every rank holds 20 client slots; a step is one client-sharded round over all
N·20 slots (every round form of feddct_amd/comm.py and dist.py is timed, see
``multi_gpu``); value = all ranks' algorithmic bytes / max-over-ranks time of
the fastest form whose result is bit-identical to the single-GPU reduction.

Also reported on the same JSON line: the roofline of the reduce kernel
(HIP-event launch time vs the 8 TB/s HBM3E peak), the CPU baseline (the
reference loop restated in torch, oracle/torch_mirror.py, on this host's
cores; rank 0, N=1 only), parity of the output against the reference's
committed SHA-256 digest, and the host-inclusive rate (pinned H2D + kernel +
D2H).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from feddct_amd import _lib, slab  # noqa: E402  (loads libfedagg.so or fails loudly)
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
LAYOUT = "wrn16_8_c10"
N_CLIENTS = 20
METRIC = "device-resident GB/s: 20-client wide_resnet16_8 weighted param reduction"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_launches(fn, steps, warmup, sync_group=None, per_launch=None):
    """W untimed steps, then exactly K timed steps between two barriers and
    device syncs; HIP events on the current stream bracket the K steps.
    ``per_launch`` (a list): also an event between consecutive steps, so the
    K per-step durations (which sum to the total) are reported — a clock ramp
    shows up as a trend in them."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if sync_group is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True)
          for _ in range(steps + 1 if per_launch is not None else 2)]
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        fn()
        if per_launch is not None:
            ev[i + 1].record()
    ev[-1].record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if sync_group is not None:
        dist.barrier()
    if per_launch is not None:
        per_launch[:] = [ev[i].elapsed_time(ev[i + 1]) / 1e3 for i in range(steps)]
    return ev[0].elapsed_time(ev[-1]) / 1e3 / steps, wall / steps


def launch_stats(ts):
    """min / median / max / first / last of per-step seconds, in µs."""
    if not ts:
        return None
    s = sorted(ts)
    return {"min_us": round(s[0] * 1e6, 2), "median_us": round(s[len(s) // 2] * 1e6, 2),
            "max_us": round(s[-1] * 1e6, 2), "first_us": round(ts[0] * 1e6, 2),
            "last_us": round(ts[-1] * 1e6, 2), "n": len(ts)}


ABORT_RC = 3   # exit status of a run ended by a phase deadline (never 0)


class PhaseDeadline:
    """``with PhaseDeadline(name, seconds, on_abort):`` — if the block is
    still running after ``seconds`` (a collective that never completes),
    ``on_abort(name)`` runs on a timer thread (it prints the flagged line) and
    the process then exits with ABORT_RC, so the driver sees a failed run and
    not a number from a hung job."""

    def __init__(self, name, seconds, on_abort):
        self.name, self.seconds, self.on_abort = name, seconds, on_abort

    def _fire(self):
        try:
            self.on_abort(self.name)
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(ABORT_RC)

    def __enter__(self):
        import threading
        self.timer = threading.Timer(self.seconds, self._fire)
        self.timer.daemon = True
        self.timer.start()
        return self

    def __exit__(self, *exc):
        self.timer.cancel()
        return False


def gpu_state_under_load(fn, max_s=20.0):
    """Clocks, power and temperatures of this GPU sampled by `rocm-smi` (a
    child process: it reads the driver's sysfs) WHILE `fn` — the headline's
    reduce — keeps the GPU busy, so the line says at what clocks its number
    was taken (box-to-box the same tree measured 133.5-144 us per launch,
    DESIGN §4).  None when the tool is absent; a dict with "error" when it
    fails or outlives `max_s`."""
    import shutil
    import subprocess
    exe = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi"
                                       if os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if exe is None:
        return None
    idx = torch.cuda.current_device()
    try:
        proc = subprocess.Popen([exe, "-d", str(idx), "--showclocks", "--showpower",
                                 "--showtemp", "--showmemuse", "--showserial", "--json"],
                                stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    except OSError as e:
        return {"error": repr(e)}
    t0 = time.perf_counter()
    launches = 0
    while proc.poll() is None and time.perf_counter() - t0 < max_s:
        for _ in range(20):
            fn()
        launches += 20
        torch.cuda.synchronize()
    if proc.poll() is None:
        proc.kill()
        proc.communicate()
        return {"error": f"rocm-smi still running after {max_s:.0f} s"}
    st = parse_smi(proc.communicate()[0])
    if "error" not in st:
        st = {"sampled_during": f"{launches} headline launches", **st}
    return st


def gpu_state_idle(max_s=20.0):
    """The same fields before this process allocates anything: memory
    already allocated on the GPU by others (a box measured with 81 % of its
    VRAM taken while idle ran this bench 5-7 % slower than boxes at 1 %)."""
    import shutil
    import subprocess
    exe = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi"
                                       if os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if exe is None:
        return None
    idx = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        r = subprocess.run([exe, "-d", str(idx), "--showclocks", "--showpower", "--showtemp",
                            "--showmemuse", "--json"], capture_output=True, text=True,
                           timeout=max_s)
    except (OSError, subprocess.TimeoutExpired) as e:
        return {"error": repr(e)}
    st = parse_smi(r.stdout)
    st.pop("serial", None)
    return st


def parse_smi(out: str) -> dict:
    """The fields gpu_state_under_load reports from `rocm-smi --json` text
    (warning lines before the JSON are skipped)."""
    import re
    try:
        card = next(iter(json.loads(out[out.index("{"):]).values()))
    except (ValueError, StopIteration) as e:
        return {"error": f"unparsed rocm-smi output: {e!r}"}

    def num(key_part):
        for k, v in card.items():
            if key_part.lower() in k.lower():
                m = re.search(r"[-+]?\d+(\.\d+)?", str(v))
                if m:
                    return float(m.group(0))
        return None
    return {"sclk_mhz": num("sclk clock speed"),
            "mclk_mhz": num("mclk clock speed"), "fclk_mhz": num("fclk clock speed"),
            "socket_power_w": num("Current Socket Graphics Package Power"),
            "junction_c": num("Temperature (Sensor junction)"),
            "memory_c": num("Temperature (Sensor memory)"),
            "vram_used_pct": num("GPU Memory Allocated"),
            "serial": next((str(v) for k, v in card.items() if "serial" in k.lower()), None)}


def digest_of(layout, out32, out64, prefix=""):
    """SHA-256 of the keys under ``prefix`` (stripped), as tests/golden does."""
    import hashlib
    f = out32.cpu().numpy()
    i = out64.cpu().numpy()
    h = hashlib.sha256()
    for s in layout.slots:
        if not s.key.startswith(prefix):
            continue
        src = i if s.kind == "i64" else f
        h.update(s.key[len(prefix):].encode())
        h.update(np.ascontiguousarray(src[s.offset:s.offset + s.numel]).tobytes())
    return h.hexdigest()


def ulp_dist(a: torch.Tensor, b: torch.Tensor) -> int:
    ia = a.view(torch.int32).to(torch.int64)
    ib = b.view(torch.int32).to(torch.int64)
    ia = torch.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return int((ia - ib).abs().max().item())


ULP_BUCKETS = ((0, 0), (1, 1), (2, 2), (3, 4), (5, 8), (9, 16), (17, None))


def ulp_hist(a: torch.Tensor, b: torch.Tensor) -> dict:
    """Histogram of per-element ULP distances (SURVEY.md §8 e1 asks for one:
    the client-sharded sum is re-associated, so it is not bit-exact)."""
    ia = a.view(torch.int32).to(torch.int64)
    ib = b.view(torch.int32).to(torch.int64)
    ia = torch.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    d = (ia - ib).abs()
    out = {}
    for lo, hi in ULP_BUCKETS:
        m = d >= lo if hi is None else (d >= lo) & (d <= hi)
        out[f"{lo}+" if hi is None else (str(lo) if lo == hi else f"{lo}-{hi}")] = int(m.sum().item())
    return out


def pmc_traffic(n_gpus):
    """HBM bytes per launch of the reduce kernel, with where they come from.
    PMC counters cannot be read from inside the timed process (rocprofv3
    --pmc is its own run), so this is the committed summary of separate
    FETCH_SIZE / WRITE_SIZE passes over THIS bench command's reduce launches
    (tools/gpu_profile.sh -> profiles/reduce_pmc.json, gfx950 FETCH_SIZE x2
    correction applied) — returned with its source and that run's average
    launch time, so the line shows what the counters were taken on."""
    path = os.path.join(ROOT, "profiles", "reduce_pmc.json")
    if n_gpus != 1 or not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == f"{LAYOUT}/n{N_CLIENTS}":
            return d.get("hbm_bytes_per_launch"), {
                "source": "profiles/reduce_pmc.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                          "passes (separate runs) of bench.py --kernel-only",
                "profile_kernel_avg_us": round(d["avg_ns"] / 1e3, 2) if "avg_ns" in d else None,
                "profile_date_utc": d.get("date_utc"), "profile_host": d.get("host"),
                "profile_gpu": d.get("gpu"), "profile_tree": d.get("tree"),
                "note": "measured in a separate profiler run (counters cannot be read from "
                        "inside the timed process), not in this run",
                "traffic_over_algorithmic": round(d["hbm_bytes_per_launch"]
                                                  / d["algorithmic_bytes_per_launch"], 4)
                if d.get("algorithmic_bytes_per_launch") else None}
    except Exception:
        pass
    return None, None


def cpu_quota() -> dict:
    """The process's CPU share as the kernel enforces it: the cgroup CPU
    quota (v2 cpu.max or v1 cfs_quota_us / cfs_period_us), the cpuset and the
    affinity mask (a container sees the whole machine's CPUs in both of the
    latter, the quota is what it gets)."""
    out = {"affinity_cpus": len(os.sched_getaffinity(0)), "host_cpus": os.cpu_count()}

    def rd(path):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return None
    v2 = rd("/sys/fs/cgroup/cpu.max")
    if v2:
        q, _, per = v2.partition(" ")
        out["cgroup"] = f"v2 cpu.max = {v2}"
        if q != "max":
            out["quota_cpus"] = round(int(q) / int(per or 100000), 2)
    else:
        q = rd("/sys/fs/cgroup/cpu/cpu.cfs_quota_us")
        per = rd("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
        if q is not None:
            out["cgroup"] = f"v1 cfs_quota_us = {q}, cfs_period_us = {per}"
            if int(q) > 0 and per:
                out["quota_cpus"] = round(int(q) / int(per), 2)
    cs = rd("/sys/fs/cgroup/cpuset.cpus.effective") or rd("/sys/fs/cgroup/cpuset/cpuset.cpus")
    if cs:
        out["cpuset"] = cs
    out["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    return out


CPU_THREADS = (1, 8, 16, 32, 64)


def run_cpu_baseline(layout, manifest, clients, budget_s=25.0):
    """The reference loop (oracle/torch_mirror.py, train_fedavg.py:138-149)
    on this box's host cores, at torch intra-op thread counts 1, 8, 16, 32
    and 64: value = the BEST count's rate.  The sweep
    goes up in threads and stops once a count runs 3x slower than the best so
    far (past the CPU quota the loop collapses: r02, 256 threads on a 16-CPU
    share ran 160x slower)."""
    from oracle.torch_mirror import arithmetic_core, reference_loop, time_call

    quota = cpu_quota()
    all_cores = quota["affinity_cpus"]
    counts = [c for c in CPU_THREADS if c <= all_cores]
    Holder = _holder_class(layout)

    def to_module(f32, i64):
        m = Holder()
        fh, ih = f32.cpu(), i64.cpu()
        sd = m.state_dict()
        with torch.no_grad():
            for s in layout.slots:
                src = ih if s.kind == "i64" else fh
                sd[s.key].copy_(src[s.offset:s.offset + s.numel].view(s.shape))
        return m

    mods = [to_module(f, i) for f, i in clients]
    g = Holder()
    by_threads, skipped = {}, []
    for th in counts:
        if by_threads:
            last = by_threads[max(by_threads)][0]
            if last > 3 * min(v[0] for v in by_threads.values()):
                skipped.append(th)
                continue
        torch.set_num_threads(th)
        tl, rp = time_call(lambda: reference_loop(g, mods), 5, budget_s * 0.5 / len(counts))
        by_threads[th] = (tl, rp)
    threads = min(by_threads, key=lambda k: by_threads[k][0])
    t_loop, reps = by_threads[threads]
    torch.set_num_threads(threads)
    states = [m.state_dict() for m in mods]
    t_core, _ = time_call(lambda: arithmetic_core(states), 3, budget_s * 0.1)
    # BASELINE config 1's shape: the loop over 2 clients (beside bench's
    # cfg1_host_resident_n2 drop-in timing)
    g2 = Holder()
    t_cfg1, reps_cfg1 = time_call(lambda: reference_loop(g2, mods[:2]), 5, budget_s * 0.1)
    # BASELINE config 3's FedDCT round (train_feddct.py:34-56): the loop on
    # the main-client models, then on the proxies, 5 slots
    fd = _feddct_modules(torch.device("cuda", torch.cuda.current_device()), cpu=True)
    t_fd, reps_fd = time_call(lambda: [reference_loop(g_, ms_) for _, _, g_, ms_ in fd], 3,
                              budget_s * 0.2)
    del fd
    # the same on one thread (SURVEY.md §8 d asks for both)
    torch.set_num_threads(1)
    t_loop1, reps1 = by_threads[1] if 1 in by_threads else time_call(
        lambda: reference_loop(g, mods), 3, budget_s * 0.3)
    t_core1, _ = time_call(lambda: arithmetic_core(states), 3, budget_s * 0.1)
    torch.set_num_threads(threads)
    nbytes = layout.algorithmic_bytes(len(clients))
    return {"value": round(nbytes / t_loop / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": (f"full reference loop (K·N state_dict rebuilds + stack/mean + "
                       f"load_state_dict + broadcast) over the same {len(clients)}-client "
                       f"{LAYOUT} state, median of {reps} runs, {t_loop * 1e3:.1f} ms/run; "
                       f"arithmetic-only stack+mean {t_core * 1e3:.1f} ms "
                       f"({nbytes / t_core / 1e9:.2f} GB/s)"),
            "loop_ms": round(t_loop * 1e3, 2), "core_ms": round(t_core * 1e3, 2),
            "one_thread": {"loop_ms": round(t_loop1 * 1e3, 2), "core_ms": round(t_core1 * 1e3, 2),
                           "loop_GBps": round(nbytes / t_loop1 / 1e9, 3), "runs": reps1},
            "cfg1_n2": {"loop_ms": round(t_cfg1 * 1e3, 2), "runs": reps_cfg1},
            "cfg3_feddct_n5": {"loop_ms": round(t_fd * 1e3, 2), "runs": reps_fd},
            "loop_ms_by_threads": {str(k): round(v[0] * 1e3, 2) for k, v in by_threads.items()},
            "threads_skipped": skipped,
            "best_threads": threads,
            "threads_note": ("torch intra-op threads swept over 1/8/16/32/64 (stopping once a "
                             "count runs 3x slower than the best); value = the best count"),
            "cpu_quota": quota,
            "host_cpus": os.cpu_count(), "affinity_cpus": all_cores, "cpu": _cpu_model()}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_inclusive(layout, clients, reducer_dev, out32, out64, reps=3):
    """Client buckets in pinned host memory, result back to host.
    serial:    H2D of N·B, one kernel, D2H of B, one stream;
    pipelined: feddct_amd/pipeline.py (column chunks, H2D / reduce / D2H
               overlapped on two copy streams), result to the global only,
               and with the broadcast into all N client buckets too
               (tapered chunks; pipelined_even8: r02's 8 even chunks; the
               broadcast fanned out on the CPU, _dma: N D2H copies per chunk);
    serial_pageable: the serial round from ordinary (pageable) host tensors
               and into a pageable result (SURVEY.md §8 d asks for both)."""
    from feddct_amd.pipeline import HostPipeline
    n = len(clients)
    host = [(c[0].cpu().pin_memory(), c[1].cpu().pin_memory()) for c in clients]
    out_h32 = torch.empty_like(out32, device="cpu").pin_memory()
    out_h64 = torch.empty_like(out64, device="cpu").pin_memory()
    nbytes = layout.algorithmic_bytes(n)

    def serial():
        for (h32, h64), (d32, d64) in zip(host, clients):
            d32.copy_(h32, non_blocking=True)
            d64.copy_(h64, non_blocking=True)
        reducer_dev()
        out_h32.copy_(out32, non_blocking=True)
        out_h64.copy_(out64, non_blocking=True)
        torch.cuda.synchronize()

    pageable = [(c[0].cpu(), c[1].cpu()) for c in clients]
    out_p32 = torch.empty_like(out32, device="cpu")
    out_p64 = torch.empty_like(out64, device="cpu")

    def serial_pageable():
        for (h32, h64), (d32, d64) in zip(pageable, clients):
            d32.copy_(h32, non_blocking=True)
            d64.copy_(h64, non_blocking=True)
        reducer_dev()
        out_p32.copy_(out32, non_blocking=True)
        out_p64.copy_(out64, non_blocking=True)
        torch.cuda.synchronize()

    pipe = HostPipeline(layout, n, out32.device)            # tapered chunks (r03)
    pipe8 = HostPipeline(layout, n, out32.device, nchunks=8)   # r02's even cut
    h32 = [h[0] for h in host]
    h64 = [h[1] for h in host]

    def piped():
        pipe.run(h32, h64, out_h32, out_h64)

    def piped_even8():
        pipe8.run(h32, h64, out_h32, out_h64)

    def piped_bcast():          # broadcast: one D2H per chunk, CPU fan-out
        pipe.run(h32, h64, out_h32, out_h64, h32, h64)

    def piped_bcast_dma():      # broadcast: N + 1 D2H per chunk (r02)
        pipe.run(h32, h64, out_h32, out_h64, h32, h64, fanout="dma")

    res = {"source": "pinned", "algorithmic_bytes": nbytes}
    # the pipelined result is the same bits as the device-resident one
    reducer_dev()
    torch.cuda.synchronize()
    piped()
    res["pipelined_bit_exact"] = bool(torch.equal(out_h32, out32.cpu()) and
                                      torch.equal(out_h64, out64.cpu()))
    for name, fn in (("serial", serial), ("serial_pageable", serial_pageable),
                     ("pipelined", piped), ("pipelined_even8", piped_even8),
                     ("pipelined_with_broadcast", piped_bcast),
                     ("pipelined_with_broadcast_dma", piped_bcast_dma)):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        t = (time.perf_counter() - t0) / reps
        res[name] = {"ms": round(t * 1e3, 3), "GBps": round(nbytes / t / 1e9, 2)}
    res["serial_pageable"]["bit_exact"] = bool(torch.equal(out_p32, out32.cpu()) and
                                               torch.equal(out_p64, out64.cpu()))
    del pageable
    return res


def round_block(layout, clients, out32, out64, plan, extra, k=40):
    """The whole server_aggregate round (train_fedavg.py:145-149: the mean,
    the global's load, the broadcast into every client slot) on its measured
    roofline: FA_F_BCAST = the reduce launch + the
    broadcast launch.  Algorithmic bytes: reduce N*B read + B written,
    broadcast B read + N*B written, 2*(N+1)*B in all.  Also each launch's
    time inside the round (the round as two calls with events between them),
    and this box's write ceiling: a write-only probe of non-zero hashed
    register values in the broadcast's own launch shape over the client
    buckets themselves (same placement), best of three passes — so it
    overwrites the clients and runs after every measurement that needs their
    values.  Ceiling fractions: the round's reads (N+1)*B at the read
    ceiling plus its writes (N+1)*B at the write ceiling, over the round."""
    n = len(clients)
    B = layout.state_bytes()
    red_bytes = layout.algorithmic_bytes(n)
    bc_bytes = (n + 1) * B
    bred = Reducer(layout, clients, out32, out64, flags=_lib.FA_F_BCAST, plan=plan)
    t_round, _ = timed_launches(bred, k, 5)
    # each launch inside the round
    red = Reducer(layout, clients, out32, out64, plan=plan)
    bco = Reducer(layout, clients, out32, out64, flags=_lib.FA_F_BCAST_ONLY, plan=plan)
    for _ in range(3):
        red()
        bco()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * k + 1)]
    ev[0].record()
    for i in range(k):
        red()
        ev[2 * i + 1].record()
        bco()
        ev[2 * i + 2].record()
    ev[-1].synchronize()
    tr = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e-3 for i in range(k))[k // 2]
    tb = sorted(ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) * 1e-3 for i in range(k))[k // 2]
    t_alone, _ = timed_launches(bco, k, 5)
    # the write ceiling over the client buckets (their values are gone after)
    dst = _lib.ptr_array([c[0].data_ptr() for c in clients])
    numel = clients[0][0].numel()
    seed = [0]

    def write_probe():
        seed[0] += 1
        _lib.check(_lib.lib.fa_write_probe_f32(dst, n, numel, seed[0],
                                               torch.cuda.current_stream().cuda_stream))
    tw = min(timed_launches(write_probe, k, 3)[0] for _ in range(3))
    wceil = n * numel * 4 / tw / 1e9
    rceil = extra.get("read_ceiling_GBps")
    out = {
        "us": round(t_round * 1e6, 1),
        "algorithmic_bytes": red_bytes + bc_bytes,
        "GBps": round((red_bytes + bc_bytes) / t_round / 1e9, 1),
        "frac": round((red_bytes + bc_bytes) / t_round / 1e9 / HBM_PEAK_GBS, 4),
        "reduce_in_round_us": round(tr * 1e6, 1),
        "bcast_in_round_us": round(tb * 1e6, 1),
        "bcast_alone_us": round(t_alone * 1e6, 1),
        "bcast_bytes": bc_bytes,
        "bcast_in_round_frac": round(bc_bytes / tb / 1e9 / HBM_PEAK_GBS, 4),
        "bcast_alone_frac": round(bc_bytes / t_alone / 1e9 / HBM_PEAK_GBS, 4),
        "write_ceiling_GBps": round(wceil, 1),
        "write_ceiling_probe": (f"fa_write_probe_f32: {n} x {numel} floats of hashed register "
                                "values into the client buckets, the shipped broadcast's launch "
                                "shape (1024-float parts, client groups of <= 24, sc1 nt "
                                "stores), best of 3 passes"),
    }
    if rceil:
        # the time the round's bytes take at this box's read and write ceilings
        t_ceil = (n + 1) * B / (rceil * 1e9) + (n + 1) * B / (wceil * 1e9)
        tb_ceil = B / (rceil * 1e9) + n * B / (wceil * 1e9)
        out["vs_box_ceilings"] = {
            "round": round(t_ceil / t_round, 4),
            "bcast_in_round": round(tb_ceil / tb, 4),
            "bcast_alone": round(tb_ceil / t_alone, 4),
            "round_vs_copy": round((red_bytes + bc_bytes) / t_round / 1e9
                                   / extra["copy_ceiling_GBps"], 4),
            "note": "ceiling time = reads at read_ceiling_GBps + writes at write_ceiling_GBps"}
    # the round's PMC traffic per launch, from its committed profiler run
    # (tools/gpu_round_pmc.sh -> profiles/round_pmc.json; separate passes, as
    # roofline.traffic)
    path = os.path.join(ROOT, "profiles", "round_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
        kt = {}
        for k in d.get("kernels", []):
            tot = k["fetch_bytes_x2"] + k["write_bytes"]
            kind = "reduce" if "reduce_kernel" in k["kernel"] else "bcast"
            kt[kind] = {"hbm_bytes": int(tot), "over_algorithmic":
                        round(tot / k["algorithmic_bytes"], 4), "kernel": k["kernel"][:60]}
        out["traffic_pmc"] = {**kt, "source": "profiles/round_pmc.json: rocprofv3 --pmc "
                              "FETCH_SIZE (x2, gfx950) / WRITE_SIZE passes of "
                              "tools/round_prof.py round (separate runs)",
                              "profile_tree": d.get("tree")}
    except Exception:
        pass
    extra["write_ceiling_GBps"] = out["write_ceiling_GBps"]
    return out


def separate_allocations_ab(layout, clients, reducer, out32, out64, rounds=3, k=50):
    """The headline's reduce over its slab-carved buckets (slab.py, the
    product's storage) against the same values in 20 + 1 separate
    allocations (the r02 storage), interleaved in this process: on some
    boxes the separate allocations read ~8 % slower
    (profiles/r03_exp_alloc.jsonl)."""
    sep = [(c32.clone(), c64) for c32, c64 in clients]
    o32 = torch.zeros_like(out32)
    o64 = torch.zeros_like(out64)
    red = Reducer(layout, sep, o32, o64, plan=reducer.plan)
    ts = {"slab": [], "separate": []}
    for _ in range(rounds):
        ts["slab"].append(timed_launches(reducer, k, 5)[0])
        ts["separate"].append(timed_launches(red, k, 5)[0])
    med = {n: sorted(v)[len(v) // 2] for n, v in ts.items()}
    out = {f"{n}_us": round(t * 1e6, 2) for n, t in med.items()}
    out["separate_over_slab"] = round(med["separate"] / med["slab"], 4)
    out["bit_equal"] = bool(torch.equal(o32.view(torch.int32), out32.view(torch.int32))
                            and torch.equal(o64, out64))
    del sep, red
    return out


def other_configs(dev, steps=100, warmup=20):
    """The other BASELINE.json configs on this GPU (device-resident), each
    checked against the reference digests where they exist:
    cfg3 FedDCT sf4 C10, 5 slots, main + proxy (two launches), working set
      rotated over 2 copies (> the 256 MiB Infinity Cache);
    cfg4 FedProx C100, 20 clients, client-size-weighted (extension);
    cfg5 FedDCT sf4 C100, 24 slots, main + proxy, all on one GPU."""
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dig = json.load(f)
    res = {}

    def run(name, parts, rot, digests):
        """parts: [(manifest names joined in ONE layout, n, weights)] — a
        FedDCT slot's main + proxy share one bucket (aggregate._Pair), so a
        round is one launch."""
        from feddct_amd.workload import joint_manifest
        sets = []
        for r in range(rot):
            reds = []
            for names, n, w in parts:
                mans = [load_manifest(x) for x in names]
                prefixes = ("0.", "1.") if len(names) > 1 else ("",)
                man = joint_manifest(mans, prefixes) if len(names) > 1 else mans[0]
                lay = BucketLayout.from_manifest(man)
                # placed as the drop-in places a round (aggregate.py: a new
                # slab sized for the N clients + the global, slab.expecting)
                slab.release()
                with slab.expecting(n + 1):
                    cl = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
                    o32 = slab.carve(cl[0][0].numel(), torch.float32, dev)
                o64 = torch.zeros_like(cl[0][1])
                reds.append((names, prefixes, lay, n, Reducer(lay, cl, o32, o64, weights=w),
                             o32, o64))
            sets.append(reds)
        k = [0]

        def step():
            for r in sets[k[0] % rot]:
                r[4]()
            k[0] += 1
        # steady state, as the headline's defaults (a 44 us launch timed 20
        # times after 3 warm-ups read ~1.5 us slow per launch: the first
        # launch after the sync pays the ramp)
        t, _ = timed_launches(step, steps, warmup)
        nbytes = sum(r[2].algorithmic_bytes(r[3]) for r in sets[0])
        out = {"GBps": round(nbytes / t / 1e9, 1), "us_per_step": round(t * 1e6, 1),
               "algorithmic_bytes": nbytes, "rotated_sets": rot,
               "launches_per_step": len(sets[0])}
        if digests:
            ok = True
            for names, prefixes, lay, n, _, o32, o64 in sets[0]:
                for nm, pf in zip(names, prefixes):
                    if digests[nm].startswith("weighted/"):
                        ok &= weighted_digest_check(digests[nm][9:], lay, o32, o64)["bit_exact"]
                    else:
                        ok &= digest_of(lay, o32, o64, pf) == dig[digests[nm]]
            out["bit_exact_vs_reference_digest" if not any(
                d.startswith("weighted/") for d in digests.values())
                else "bit_exact_vs_weighted_definition_digest"] = bool(ok)
        # the whole round: reduce + broadcast over the
        # same rotated sets, as the product launches it (two launches; the
        # single-pass form measured slower on every layout, r04, and was
        # removed in r05: DESIGN §4.2)
        rb_bytes = sum(r[2].algorithmic_bytes(r[3]) + (r[3] + 1) * r[2].state_bytes()
                       for r in sets[0])
        rsets = [[Reducer(lay, red._keep[0], o32, o64,
                          weights=None if red.w is None else list(red.w),
                          flags=_lib.FA_F_BCAST, plan=red.plan)
                  for names, prefixes, lay, n, red, o32, o64 in reds] for reds in sets]
        kr = [0]

        def rstep():
            for r in rsets[kr[0] % rot]:
                r()
            kr[0] += 1
        tr, _ = timed_launches(rstep, steps, warmup)
        out["round_us"] = round(tr * 1e6, 1)
        out["round_frac"] = round(rb_bytes / tr / 1e9 / HBM_PEAK_GBS, 4)
        out["round_algorithmic_bytes"] = rb_bytes
        res[name] = out

    run("cfg3_feddct_c10_n5", [(("wrnsl16_8_sf4_c10_main", "wrnsl16_8_sf4_c10_proxy"), 5, None)], 2,
        {"wrnsl16_8_sf4_c10_main": "feddct/wrnsl16_8_sf4_c10_main/n5",
         "wrnsl16_8_sf4_c10_proxy": "feddct/wrnsl16_8_sf4_c10_proxy/n5"})
    from feddct_amd.aggregate import client_weights as weights_from_sizes
    sizes = [2500 + 97 * ((7 * i) % 11) for i in range(20)]  # quantity-skewed shards
    run("cfg4_fedprox_c100_n20_weighted", [(("wrn16_8_c100",), 20, weights_from_sizes(sizes))],
        1, {"wrn16_8_c100": "weighted/wrn16_8_c100/n20/cfg4_sizes"})
    run("cfg5_feddct_c100_n24_one_gpu", [(("wrnsl16_8_sf4_c100_main", "wrnsl16_8_sf4_c100_proxy"),
                                          24, None)], 1,
        {"wrnsl16_8_sf4_c100_main": "feddct/wrnsl16_8_sf4_c100_main/n24",
         "wrnsl16_8_sf4_c100_proxy": "feddct/wrnsl16_8_sf4_c100_proxy/n24"})
    # r03: the reference's other FedDCT sweep layouts,
    # rotated over enough sets that every step misses the 256 MiB MALL
    for tag, sf, n, rot in (("resnet110sl", 4, 25, 4), ("wrnsl16_8", 32, 3, 6)):
        nm = f"{tag}_sf{sf}_c100"
        run(f"sweep_{nm}_n{n}", [((nm + "_main", nm + "_proxy"), n, None)], rot,
            {nm + "_main": f"feddct/{nm}_main/n{n}", nm + "_proxy": f"feddct/{nm}_proxy/n{n}"})
        res[f"sweep_{nm}_n{n}"].update(scalar_share(dev, nm, n, steps, warmup))
    for v in res.values():
        v["roofline_frac"] = round(v["GBps"] / HBM_PEAK_GBS, 4)
    return res


def scalar_share(dev, name, n, steps, warmup):
    """Where a layout's time goes: its scalar tiles (ILP-4 tails, M == 1 and
    int64 keys: one thread per element walking the clients) and its vector
    tiles, each launched alone over the same clients."""
    from feddct_amd.workload import joint_manifest
    mans = [load_manifest(name + "_main"), load_manifest(name + "_proxy")]
    lay = BucketLayout.from_manifest(joint_manifest(mans))
    cl = make_clients(lay, list(zip(mans, ("0.", "1."))), range(n), dev)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    info, tiles = _lib.build_tiles_host(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    cols = int(tiles[tiles[:, 2] != 0][:, 1].sum())
    out = {"scalar_tiles": int(info["ntiles_tail"]), "vector_tiles": int(info["ntiles_cascade"]),
           "scalar_columns": cols, "packed_scalar_tiles": -(-cols // 64),
           "scalar_elems_frac": round(info["tail_elems"] / max(1, info["tail_elems"]
                                                                + info["cascade_elems"]), 5)}
    for part, sel in (("scalar_tiles_alone_us", tiles[:, 2] != 0),
                      ("vector_tiles_alone_us", tiles[:, 2] == 0)):
        plan = _lib.Plan(None, lay.f32_numel, None, lay.i64_numel, 0, tiles=tiles[sel])
        t, _ = timed_launches(Reducer(lay, cl, o32, o64, plan=plan), steps, warmup)
        out[part] = round(t * 1e6, 2)
    return out


def cfg5_sharded(dev, world, rank, group, steps, ncomm=None, chain_chunks=16):
    """BASELINE config 5 on the N GPUs of this run: FedDCT sf4 C100, 24 slots
    (main + proxy in one joint bucket), slots sharded contiguously over the
    ranks (3 per GPU at N=8).  Timed as rounds: the chained exact round
    (native and torch.distributed; result on the last rank), the striped
    exact round (result on rank 0) and e1 (re-associated; rank 0).  Every
    exact result is checked bit-for-bit against the reference's digests on
    the rank that holds it."""
    from feddct_amd.dist import ChainAggregator, ShardedAggregator, StripedAggregator, shard_range
    from feddct_amd.workload import joint_manifest
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dig = json.load(f)
    names = ("wrnsl16_8_sf4_c100_main", "wrnsl16_8_sf4_c100_proxy")
    mans = [load_manifest(x) for x in names]
    prefixes = ("0.", "1.")
    lay = BucketLayout.from_manifest(joint_manifest(mans, prefixes))
    n = 24
    lo, hi = shard_range(n, world, rank)
    cl = make_clients(lay, list(zip(mans, prefixes)), range(lo, hi), dev)
    l32, l64 = [c[0] for c in cl], [c[1] for c in cl]
    o32 = torch.zeros(max(lay.f32_numel, 64), dtype=torch.float32, device=dev)
    o64 = torch.zeros(max(lay.i64_numel, 1), dtype=torch.int64, device=dev)
    nbytes = lay.algorithmic_bytes(n)
    last = world - 1

    def tmax(fn, k, w):
        t, _ = timed_launches(fn, k, w, sync_group=group)
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def exact_on(r, b32, b64):
        ok = [False]
        if rank == r:
            ok = [all(digest_of(lay, b32, b64, pf) == dig[f"feddct/{nm}/n24"]
                      for nm, pf in zip(names, prefixes))]
        dist.broadcast_object_list(ok, src=r, group=group)
        return bool(ok[0])

    out = {"slots": n, "slots_per_gpu": hi - lo, "algorithmic_bytes": nbytes}

    def mode(name, make, root, k, exact, model=None):
        try:
            b32, b64 = torch.zeros_like(o32), torch.zeros_like(o64)
            t = tmax(make(b32, b64), k, 2)
            r = {"ms": round(t * 1e3, 4), "GBps": round(nbytes / t / 1e9, 2),
                 "result_on": f"rank {root}"}
            if model is not None:
                from feddct_amd import comm as Cm
                r["model_us"] = round(Cm.round_model(model[0], lay, counts, nchunks=model[1],
                                                     root=root)["model_us"], 1)
            if exact:
                r["bit_exact_vs_reference_digest"] = exact_on(root, b32, b64)
            out[name] = r
            return b32, b64
        except Exception as e:  # noqa: BLE001
            out[name] = {"error": repr(e)}
            return None
    counts = [b - a for a, b in (shard_range(n, world, r) for r in range(world))]
    if ncomm is not None:
        from feddct_amd import comm as Cm
        from feddct_amd.comm import (NativeAggregator, NativeChainedAggregator,
                                     NativeStripedAggregator, multi_select)
        # the default entry (r06: the cost model's exact form and chunk count
        # — the link-parallel striped round at 8 x 3; r05: chained)
        droot = max(r for r in range(world) if counts[r] > 0)
        form, fk, _ = multi_select(counts, layout=lay, detail=True)
        mode("default_native", lambda b32, b64: NativeAggregator(
            lay, l32, l64, n, b32, b64, ncomm, final="reduce", root=droot).step, droot, steps,
            True, model=(Cm.MODE_IDS[form], fk))
        if "default_native" in out and "ms" in out["default_native"]:
            out["default_native"].update(form=form, nchunks=fk)
        mode("chained_native", lambda b32, b64: NativeChainedAggregator(
            lay, l32, l64, n, b32, b64, ncomm, nchunks=chain_chunks, final="reduce",
            root=last).step, last, steps, True, model=(Cm.FA_MODE_CHAINED, chain_chunks))
        for k in (1, 4):
            mode(f"striped_native_c{k}", lambda b32, b64, k=k: NativeStripedAggregator(
                lay, l32, l64, n, b32, b64, ncomm, final="reduce", root=last,
                nchunks=k).step, last, max(2, steps // 2), True, model=(Cm.FA_MODE_STRIPED, k))
    mode("chained_torch_distributed", lambda b32, b64: (lambda a: lambda: a.step(l32, l64))(
        ChainAggregator(lay, n, b32, b64, group=group, final="reduce", root=last,
                        nchunks=chain_chunks)), last, max(2, steps // 2), True)
    e2 = mode("e2_torch_distributed", lambda b32, b64: (lambda a: lambda: a.step_device(
        l32, l64))(StripedAggregator(lay, n, b32, b64, group=group, final="reduce")), 0,
        max(2, steps // 10), True)
    e1 = mode("e1_torch_distributed", lambda b32, b64: ShardedAggregator(
        lay, l32, l64, n, b32, b64, final="reduce").step, 0, steps, False)
    if rank == 0 and e1 is not None and e2 is not None:
        out["e1_torch_distributed"]["max_abs_err_vs_exact"] = float((e1[0] - e2[0]).abs().max())
        out["e1_torch_distributed"]["int64_bit_exact"] = bool(torch.equal(e1[1], e2[1]))
    # the sharding decision: the same 24 slots
    # all on ONE GPU (rank 0 generates every slot), one plain reduce launch —
    # printed beside the fastest exact multi-GPU round of this run
    one = None
    if rank == 0:
        try:
            cl_all = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
            a32, a64 = torch.zeros_like(o32), torch.zeros_like(o64)
            t1, _ = timed_launches(Reducer(lay, cl_all, a32, a64), steps, 5)
            one = {"ms": round(t1 * 1e3, 4), "GBps": round(nbytes / t1 / 1e9, 2),
                   "bit_exact_vs_reference_digest": all(
                       digest_of(lay, a32, a64, pf) == dig[f"feddct/{nm}/n24"]
                       for nm, pf in zip(names, prefixes))}
            del cl_all
        except Exception as e:  # noqa: BLE001
            one = {"error": repr(e)}
    exact = {k: v["ms"] for k, v in out.items() if isinstance(v, dict) and "ms" in v
             and v.get("bit_exact_vs_reference_digest")}
    if one is not None:
        out["one_gpu_all_slots"] = one
        if exact:
            best = min(exact, key=exact.get)
            out["decision"] = {
                "fastest_exact_multi_gpu": best, "multi_gpu_ms": exact[best],
                "one_gpu_ms": one.get("ms"),
                "rule": "slots already on one GPU: keep them there while N*B fits its HBM "
                        "(one launch); slots trained on W GPUs: the exact sharded round, "
                        "never a gather of (W-1)/W*N*B over xGMI (DESIGN §8)"}
    return out


def cfg1_host_resident(dev, reps=5):
    """BASELINE config 1's shape — FedAvg, 2 clients, wide_resnet16_8 C10,
    modules in HOST memory — through the drop-in server_aggregate (pinned
    arenas, chunked H2D / reduce / D2H incl. the broadcast back into both
    clients), checked against the reference digest."""
    from feddct_amd.aggregate import server_aggregate
    man = load_manifest("wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    Holder = _holder_class(layout)
    n = 2
    dev_clients = make_clients(layout, man, range(n), dev)
    mods = []
    for f32, i64 in dev_clients:
        m = Holder()
        sd = m.state_dict()
        with torch.no_grad():
            for s in layout.slots:
                src = i64 if s.kind == "i64" else f32
                sd[s.key].copy_(src[s.offset:s.offset + s.numel].view(s.shape).cpu())
        mods.append(m)
    snap = [{k: v.clone() for k, v in m.state_dict().items()} for m in mods]
    g = Holder()
    server_aggregate(g, mods)  # binds the pinned arenas
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        want = json.load(f)["fedavg/wrn16_8_c10/n2"]
    import hashlib
    h = hashlib.sha256()
    for k, v in g.state_dict().items():
        h.update(k.encode())
        h.update(v.numpy().tobytes())
    ok = h.hexdigest() == want
    ts = []
    for _ in range(reps):
        for m, sn in zip(mods, snap):  # restore the inputs (the round broadcast over them)
            m.load_state_dict(sn)
        t0 = time.perf_counter()
        server_aggregate(g, mods)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    t = ts[len(ts) // 2]
    return {"server_aggregate_ms": round(t * 1e3, 2), "bit_exact_vs_reference_digest": bool(ok),
            "note": "host-resident modules, pinned arenas, PCIe H2D/D2H incl. broadcast"}


def exact_modes(layout, manifest, clients, out32, out64, world, group, dev, nbytes_rank,
                steps, ncomm=None):
    """N>1: the exact column-striped mode (feddct_amd/dist.py),
    with device-resident client shards and with host ingress."""
    from feddct_amd.dist import StripedAggregator
    from feddct_amd.workload import fill_client
    n_total = N_CLIENTS * world

    def timed_max(fn, k, w):
        t, _ = timed_launches(fn, k, w, sync_group=group)
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    s32, s64 = torch.zeros_like(out32), torch.zeros_like(out64)
    sagg = StripedAggregator(layout, n_total, s32, s64, group=group, final="reduce")
    lc32, lc64 = [c[0] for c in clients], [c[1] for c in clients]
    ts = timed_max(lambda: sagg.step_device(lc32, lc64), steps, 2)
    striped = {"mode": "column-striped exact (grouped P2P stripe exchange over RCCL)",
               "ms_per_step": round(ts * 1e3, 3),
               "GBps": round(nbytes_rank * world / ts / 1e9, 2)}
    x32 = x64 = None
    if ncomm is not None:  # the same exact round through the C ABI (fa_reduce_striped)
        from feddct_amd.comm import NativeStripedAggregator
        x32, x64 = torch.zeros_like(out32), torch.zeros_like(out64)
        xagg = NativeStripedAggregator(layout, lc32, lc64, n_total, x32, x64, ncomm,
                                       final="reduce")
        tx = timed_max(xagg.step, steps, 2)
        striped["native"] = {"ms_per_step": round(tx * 1e3, 3),
                             "GBps": round(nbytes_rank * world / tx / 1e9, 2)}
        del xagg
    # host ingress (the north_star's CPU-tensor clients): each GPU uploads only
    # ITS column stripe of every client over its own PCIe link, reduces it
    # exactly, the stripes meet on the root
    h32, h64 = torch.zeros_like(out32), torch.zeros_like(out64)
    hagg = StripedAggregator(layout, n_total, h32, h64, group=group, final="reduce")
    lo, hi = hagg.lo, hagg.hi
    scratch32, scratch64 = torch.zeros_like(out32), torch.zeros_like(out64)
    stripes, host64 = [], []
    for c in range(n_total):
        fill_client(layout, manifest, scratch32, scratch64, c)
        stripes.append(scratch32[lo:hi].cpu().pin_memory())
        host64.append(scratch64.cpu().pin_memory())
    th = timed_max(lambda: hagg.step_host(stripes, host64), 3, 1)
    striped_host = {"mode": "column-striped exact, host ingress (stripe-only H2D per GPU)",
                    "ms_per_step": round(th * 1e3, 3),
                    "GBps": round(nbytes_rank * world / th / 1e9, 2),
                    "H2D_bytes_per_gpu": int((hi - lo) * 4 * n_total)}
    return striped, striped_host, (s32, s64, h32, h64, x32, x64)


def _holder_class(layout):
    class Holder(torch.nn.Module):
        def __init__(self):
            super().__init__()
            for s in layout.slots:
                parts = s.key.split(".")
                mod = self
                for p in parts[:-1]:
                    if p not in mod._modules:
                        mod.add_module(p, torch.nn.Module())
                    mod = mod._modules[p]
                t = torch.zeros(s.shape, dtype=s.dtype)
                if s.dtype == torch.int64:
                    mod.register_buffer(parts[-1], t)
                else:
                    mod.register_parameter(parts[-1], torch.nn.Parameter(t))
    return Holder


def _param_module(layout, dev, seed):
    """An nn.Module with ``layout``'s state_dict, BN running stats and int64
    counters as buffers (as in the reference models), parameters filled
    from a seeded generator."""
    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            for sl in layout.slots:
                parts = sl.key.split(".")
                mod = self
                for q in parts[:-1]:
                    if q not in mod._modules:
                        mod.add_module(q, torch.nn.Module())
                    mod = mod._modules[q]
                t = torch.zeros(sl.shape, dtype=sl.dtype)
                if sl.dtype == torch.int64 or parts[-1].startswith("running_"):
                    mod.register_buffer(parts[-1], t)
                else:
                    mod.register_parameter(parts[-1], torch.nn.Parameter(t))
    m = M().to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    with torch.no_grad():
        for p_ in m.parameters():
            p_.copy_(torch.randn(p_.shape, generator=g, device=dev) * 0.05)
    return m


def next_rows(dev, steps=30):
    """SURVEY.md §8 f3/f4 measured beside the reference's own code on this box.

    f3: the FedProx proximal term sum_k ||w_k - w_t,k||_2 and its backward
    (train_fedprox.py:113-116), wrn16_8 C100 client vs global: ours (arenas,
    prox_partials + prox_finish forward, prox_grad backward) vs the
    reference's per-parameter loop on torch-ROCm on the same GPU; kernel
    roofline over the algorithmic bytes (forward reads both models' P
    parameters, backward reads both and writes both gradients: 24 B/param).
    f4: the per-round checkpoint save (train_fedavg.py:421-442,
    utils/metric.py:9-14) of the GPU global model, bucket DMA vs
    torch.save(model.state_dict())."""
    import tempfile
    from feddct_amd.checkpoint import save_checkpoint
    from feddct_amd.prox import proximal_term
    man = load_manifest("wrn16_8_c100")
    layout = BucketLayout.from_manifest(man)
    client, glob = _param_module(layout, dev, 1), _param_module(layout, dev, 2)
    P = sum(p_.numel() for p_ in client.parameters())

    # one step as the reference takes it (train_fedprox.py:113-136): the
    # optimizer zeroes the CLIENT's gradients (optimizer.zero_grad(), torch's
    # set_to_none default); the global model's accumulate step after step
    def ours():
        client.zero_grad(set_to_none=True)
        proximal_term(client, glob, flat_grads=True).backward()

    def reference():
        client.zero_grad(set_to_none=True)
        pt = 0.0
        for w, w_t in zip(client.parameters(), glob.parameters()):
            pt += (w - w_t).norm(2)
        pt.backward()

    ours()
    want = sum((w - w_t).norm(2) for w, w_t in zip(client.parameters(), glob.parameters()))
    got = proximal_term(client, glob, flat_grads=True)
    t_ours, _ = timed_launches(ours, steps, 3)
    t_ref, _ = timed_launches(reference, steps, 3)
    # kernel-only: the three launches over the bound arenas
    # (4 rotated sets of client/global/grad buckets: 704 MB > the 256 MB MALL)
    term = client.__dict__["_fa_prox"][id(glob)]
    norms = torch.empty(max(1, term.plan.nseg), device=dev)
    total = torch.empty((), device=dev)
    one = torch.ones((), device=dev)
    sets = [(term.ca.f32.clone(), term.ga.f32.clone(), torch.empty_like(term.ca.f32),
             torch.empty_like(term.ga.f32)) for _ in range(4)]
    rot = [0]

    def kernels():
        a, b, ga, gb = sets[rot[0] % 4]
        rot[0] += 1
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(_lib.lib.fa_prox_norms(term.plan.handle, a.data_ptr(), b.data_ptr(),
                                          norms.data_ptr(), total.data_ptr(), st))
        _lib.check(_lib.lib.fa_prox_grad(term.plan.handle, a.data_ptr(), b.data_ptr(),
                                         norms.data_ptr(), one.data_ptr(), 1.0, ga.data_ptr(),
                                         gb.data_ptr(), st))
    t_k, _ = timed_launches(kernels, steps * 4, 4)
    # the same with two chunks per forward workgroup (r04 A/B, fa_tune_prox_cpw)
    _lib.lib.fa_tune_prox_cpw(2)
    try:
        t_k1, _ = timed_launches(kernels, steps * 4, 4)
    finally:
        _lib.lib.fa_tune_prox_cpw(0)
    del sets

    def term_only():     # the term's own forward + backward (no zero_grad)
        proximal_term(client, glob, flat_grads=True).backward()
    t_term, _ = timed_launches(term_only, steps, 3)
    kbytes = 24 * P
    f3 = {"params": P, "step_us": round(t_ours * 1e6, 1),
          "reference_loop_step_us": round(t_ref * 1e6, 1),
          "speedup_vs_reference_loop": round(t_ref / t_ours, 2),
          "kernels_us": round(t_k * 1e6, 1),
          "kernels_GBps": round(kbytes / t_k / 1e9, 1),
          "kernels_roofline_frac": round(kbytes / t_k / 1e9 / HBM_PEAK_GBS, 4),
          "kernels_two_chunks_per_wg_us": round(t_k1 * 1e6, 1),
          "term_fwd_bwd_us": round(t_term * 1e6, 1),
          "rel_err_vs_torch": float(abs(got.item() - want.item()) / abs(want.item())),
          "note": "step = the client's zero_grad (as the reference's optimizer) + the term's "
                  "fwd + bwd incl. autograd; term_fwd_bwd_us without the zero_grad; "
                  "reference = its loop on torch-ROCm"}
    # where the kernels' time goes, from the committed profiler run of this
    # leg (tools/prox_prof.sh -> profiles/r05_prox_pmc.json)
    try:
        with open(os.path.join(ROOT, "profiles", "r05_prox_pmc.json")) as f:
            d = json.load(f)
        s = d["summary"]
        f3["kernels_pmc"] = {
            "partials_us": round(d["prox_partials"]["avg_ns"] / 1e3, 2),
            "finish_us": round(d["prox_finish"]["avg_ns"] / 1e3, 2),
            "grad_us": round(d["prox_grad"]["avg_ns"] / 1e3, 2),
            "one_workgroup_floor_us": round(d["one_workgroup_floor"]["avg_ns"] / 1e3, 2),
            "partials_traffic_over_algorithmic": s["partials_traffic_over_algorithmic"],
            "partials_vs_same_shape_read_probe": s["partials_vs_same_shape_read_probe_lab"],
            "frac_without_finish": s["frac_without_finish"],
            "limiter": "the finish (one workgroup) = the one-workgroup launch floor",
            "source": "profiles/r05_prox_pmc.json", "profile_tree": d["prox_partials"].get("tree")}
    except Exception:
        pass
    # f4: checkpoint save of the bound global model
    from feddct_amd.aggregate import server_aggregate
    server_aggregate(glob, [client])  # binds glob's arena (and client's)
    d = tempfile.mkdtemp(prefix="fa_ckpt_")
    try:
        def save_ours():
            save_checkpoint({"round": 1, "arch": "wrn16_8", "state_dict": glob,
                             "best_acc1": 0.0}, False, d, "ours.pth.tar")

        def save_ref():
            torch.save({"round": 1, "arch": "wrn16_8", "state_dict": glob.state_dict(),
                        "best_acc1": 0.0}, os.path.join(d, "ref.pth.tar"))

        def wall(fn, reps=5):
            fn()
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return sorted(ts)[reps // 2]
        to, tr = wall(save_ours), wall(save_ref)
        a = torch.load(os.path.join(d, "ours.pth.tar"), weights_only=True)["state_dict"]
        b = torch.load(os.path.join(d, "ref.pth.tar"), weights_only=True)["state_dict"]
        same = list(a.keys()) == list(b.keys()) and all(torch.equal(a[k].cpu(), b[k].cpu()) for k in a)
        f4 = {"save_ms": round(to * 1e3, 2), "reference_save_ms": round(tr * 1e3, 2),
              "files_equal": bool(same), "bytes": layout.state_bytes()}
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)
    return {"f3_fedprox_proximal_term": f3, "f4_checkpoint_save": f4}


def dropin_timing(layout, clients, dev, reps=20):
    """Wall time of the drop-in ``server_aggregate(global, clients)`` on
    nn.Modules with the wrn16_8 state_dict (arena validation + one fused
    reduce/broadcast launch + stream sync), as the round loop would call it."""
    from feddct_amd.aggregate import server_aggregate
    Holder = _holder_class(layout)
    mods = []
    for f32, i64 in clients:
        m = Holder().to(dev)
        sd = m.state_dict()
        with torch.no_grad():
            for s in layout.slots:
                src = i64 if s.kind == "i64" else f32
                sd[s.key].copy_(src[s.offset:s.offset + s.numel].view(s.shape))
        mods.append(m)
    g = Holder().to(dev)
    server_aggregate(g, mods)  # first call binds the arenas
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        server_aggregate(g, mods)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    t = ts[len(ts) // 2]
    out = {"server_aggregate_ms": round(t * 1e3, 3),
           "note": "median wall incl. Python shim, arena checks, reduce + broadcast launches, "
                   "sync; gpu_round_us: the same round's two launches back to back"}
    out.update(_bound_round_gpu(t))
    return out


def _bound_round_gpu(wall_s, reps=30):
    """GPU time of the last drop-in round (the engine's bound round: its plan,
    pointer arrays and buckets), its two launches timed back to back, and the
    drop-in's wall time beyond it (host work before the launch + the sync)."""
    from feddct_amd.aggregate import engine
    e = engine()
    rb = e._round
    if rb is None:
        return {"gpu_round_us": None}
    ga = rb.arenas[0]()

    def launch():
        e._launch(rb.plan, rb.a32, rb.a64, rb.n, None, ga.f32.data_ptr(), ga.i64.data_ptr(),
                  _lib.FA_F_BCAST, rb.dev)
    tg, _ = timed_launches(launch, reps, 3)
    return {"gpu_round_us": round(tg * 1e6, 1),
            "host_share_us": round((wall_s - tg) * 1e6, 1)}


def _feddct_modules(dev, n=5, cpu=False, classes=10):
    """BASELINE config 3's slots as nn.Modules: n main-client + n proxy
    modules (wrnsl16_8 sf4 C10 state_dicts; config 5: C100, n = 24) holding
    the synthetic states, plus the two global models."""
    names = (f"wrnsl16_8_sf4_c{classes}_main", f"wrnsl16_8_sf4_c{classes}_proxy")
    out = []
    for nm in names:
        man = load_manifest(nm)
        lay = BucketLayout.from_manifest(man)
        Holder = _holder_class(lay)
        mods = []
        for f32, i64 in make_clients(lay, man, range(n), dev):
            m = Holder() if cpu else Holder().to(dev)
            sd = m.state_dict()
            with torch.no_grad():
                for sl in lay.slots:
                    src = i64 if sl.kind == "i64" else f32
                    sd[sl.key].copy_(src[sl.offset:sl.offset + sl.numel].view(sl.shape))
            mods.append(m)
        out.append((nm, lay, Holder() if cpu else Holder().to(dev), mods))
    return out


def dropin_feddct_timing(dev, reps=20, n=5, classes=10):
    """The FedDCT drop-in ``server_aggregate(g_main, g_proxy, mains, proxies)``
    (train_feddct.py:34-56) on BASELINE config 3's shape (config 5's with
    n=24, classes=100), end to end: the result is checked against the
    reference's digests, then timed."""
    from feddct_amd.feddct import server_aggregate
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dig = json.load(f)
    (nm_m, lay_m, g_m, mains), (nm_p, lay_p, g_p, proxies) = _feddct_modules(
        dev, n=n, classes=classes)
    server_aggregate(g_m, g_p, mains, proxies)
    torch.cuda.synchronize()
    import hashlib
    ok = True
    for nm, g in ((nm_m, g_m), (nm_p, g_p)):
        h = hashlib.sha256()
        for k, v in g.state_dict().items():
            h.update(k.encode())
            h.update(v.detach().cpu().numpy().tobytes())
        ok &= h.hexdigest() == dig[f"feddct/{nm}/n{n}"]
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        server_aggregate(g_m, g_p, mains, proxies)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out = {"server_aggregate_ms": round(ts[len(ts) // 2] * 1e3, 3),
           "bit_exact_vs_reference_digest": bool(ok),
           "note": f"cfg{3 if n == 5 else 5} shape: {n} slots x (main + proxy), median wall "
                   "incl. sync; gpu_round_us: the same round's two launches back to back"}
    out.update(_bound_round_gpu(ts[len(ts) // 2]))
    return out



def weighted_digest_check(case, layout, o32, o64):
    """The weighted launch's result against the committed digest of the
    build's weighted definition (tests/golden/weighted_digests.json, made by
    tests/golden/make_weighted_digests.py; the reference has no weights)."""
    with open(os.path.join(ROOT, "tests", "golden", "weighted_digests.json")) as f:
        want = json.load(f)[f"weighted/{case}"]["digest"]
    return {"vs": "weighted definition digest (tests/golden/weighted_digests.json)",
            "bit_exact": digest_of(layout, o32, o64) == want}


def torch_gpu_order_mode(layout, clients, steps=20, warmup=3, plan_flags=None):
    """The opt-in FA_ORDER_TORCH_GPU plan (torch-ROCm's own GPU
    stack(...).mean(0) order, the reference's .cuda() runs) on the cfg2
    workload: launch time and bit-exactness against torch's cuda mean of
    every key, computed here by torch itself."""
    n = len(clients)
    fl = _lib.FA_PLAN_GAPS_ARE_PADDING if plan_flags is None else plan_flags
    plan = _lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel,
                     order=_lib.FA_ORDER_TORCH_GPU, n=n, flags=fl)
    o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
    red = Reducer(layout, clients, o32, o64, plan=plan)
    t, _ = timed_launches(red, steps, warmup)
    ok = True
    for s in layout.slots:
        src = 1 if s.kind == "i64" else 0
        ref = torch.stack([c[src][s.offset:s.offset + s.numel].view(s.shape).float()
                           for c in clients], 0).mean(0)
        if s.kind == "i64":
            want = torch.zeros(s.shape, dtype=torch.int64, device=ref.device)
            want.copy_(ref)
            ok &= bool(torch.equal(o64[s.offset:s.offset + s.numel].view(s.shape), want))
        else:
            got = o32[s.offset:s.offset + s.numel].view(s.shape)
            ok &= bool(torch.equal(got.view(torch.int32), ref.view(torch.int32)))
    nb = layout.algorithmic_bytes(n)
    return {"us": round(t * 1e6, 1), "GBps": round(nb / t / 1e9, 1),
            "bit_exact_vs_torch_cuda_mean": ok}


def multi_gpu(args, world, rank, dev, group, layout, manifest, clients, out32, out64, reducer,
              nbytes_rank, extra):
    """N>1 (weak scaling: 20 client slots per GPU, slot order = rank order).
    Every round form is timed over the same K steps (max over ranks):

    * blocked (exact client shards, native fa_reduce_blocked): block sums
      where the slots lie, the few partials cut by a shard boundary relayed
      through the column-stripe owners, the owners fold — no rank-to-rank
      pipeline;
    * chained (exact client shards; native fa_reduce_chained and the
      torch.distributed ChainAggregator): the shards stay put, the cascade
      state hops rank to rank — the north_star's client-sharded partitioning
      with the reference's bits; the global state lands on the last rank (the
      chain's end; root = W-1: no extra transfer);
    * striped e2 (exact column stripes; native and torch.distributed);
    * sharded e1 (partial sums + RCCL reduce or reduce-scatter + gather to
      rank 0; re-associated, NOT bit-exact: ULP histogram reported).

    Every mode's result is compared with the exact single-GPU reduction of all
    N·20 clients on rank 0; ``value`` is the fastest BIT-EXACT mode."""
    from feddct_amd.dist import ChainAggregator, ShardedAggregator
    n_total = N_CLIENTS * world
    l32, l64 = [c[0] for c in clients], [c[1] for c in clients]
    last = world - 1
    modes = {}      # name -> {"t": s, "root": rank or -1, "out": (o32, o64), "exact_class": bool}

    def tmax(fn, k, w):
        t, _ = timed_launches(fn, k, w, sync_group=group)
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    # kernel-only launch time for the roofline: this rank's 20-client reduce
    # (first, so a run cut short by a phase deadline still has it)
    kred = Reducer(layout, clients, torch.zeros_like(out32), torch.zeros_like(out64),
                   flags=_lib.FA_F_SUM_ONLY, plan=reducer.plan)
    t_kernel, _ = timed_launches(kred, max(10, args.steps // 2), 3)
    del kred

    deadline_s = float(os.environ.get("FA_BENCH_PHASE_DEADLINE_S", "150"))

    def abort_run(phase):
        """A phase that outlives its deadline (a collective that never
        completes) ends the run on every rank — each rank's own timer, same
        deadline — instead of leaving the job hung until the launcher's limit.
        Rank 0 first prints the line from the forms that finished, flagged
        (parity unchecked, the phase named); PhaseDeadline then exits with
        ABORT_RC."""
        import faulthandler
        log(f"[rank {rank}] phase '{phase}' exceeded {deadline_s:.0f} s; stacks follow")
        faulthandler.dump_traceback(all_threads=True)
        if rank == 0:
            done = {n: m for n, m in modes.items() if "t" in m}
            cands = [n for n in done if done[n]["exact_class"]] or list(done)
            extra["modes"] = {n: ({"ms_per_step": round(m["t"] * 1e3, 4),
                                   "GBps": round(nbytes_rank * world / m["t"] / 1e9, 2),
                                   "bit_exact": None} if "t" in m else {"error": m["error"]})
                              for n, m in modes.items()}
            extra["aborted"] = {"phase": phase, "deadline_s": deadline_s,
                                "note": "phase did not finish on every rank; results unchecked"}
            extra["headline_not_verified_exact"] = True
            if cands:
                best = min(cands, key=lambda n: done[n]["t"])
                extra["selected_mode"] = best
                print(json.dumps(build_line(args, world, nbytes_rank, layout.state_bytes(),
                                            done[best]["t"], t_kernel, extra)), flush=True)

    def phase(name):
        return PhaseDeadline(name, deadline_s, abort_run)

    counts = [N_CLIENTS] * world

    def run_mode(name, make, root, exact_class, steps=None, warm=None, model=None):
        """``model``: (FA_MODE_*, nchunks) of a native form — its modelled
        time (fa_round_model, the same root) goes beside the measured one,
        and one extra round runs profiled (fa_comm_set_profile: the exchange
        and the kernels on each stream, r06 VERDICT r05 next 4)."""
        log(f"[rank {rank}] {name}")
        try:
            with phase(name):
                o32, o64 = torch.full_like(out32, float("nan")), torch.zeros_like(out64)
                fn = make(o32, o64)
                t = tmax(fn, steps or args.steps, args.warmup if warm is None else warm)
            modes[name] = {"t": t, "root": root, "out": (o32, o64), "exact_class": exact_class}
            if model is not None and ncomm is not None:
                from feddct_amd import comm as Cm
                modes[name]["model_us"] = round(Cm.round_model(
                    model[0], layout, counts, nchunks=model[1], root=root)["model_us"], 1)
                plan = getattr(getattr(fn, "__self__", None), "plan", None)
                if plan is not None and world > 1:
                    with phase(name + " (profiled)"):
                        ncomm.set_profile(True)
                        try:
                            fn()
                            modes[name]["profile"] = Cm.plan_profile(plan)
                        finally:
                            ncomm.set_profile(False)
                        torch.cuda.synchronize()
                        dist.barrier(group=group)
        except Exception as e:  # noqa: BLE001  (reported in the line, every rank alike)
            modes[name] = {"error": repr(e)}

    ncomm = None
    if not args.same_device:
        try:
            from feddct_amd.comm import Comm
            ncomm = Comm.from_process_group(group)
        except Exception as e:  # noqa: BLE001
            extra["native_comm_error"] = repr(e)
    try:
        extra["multi_env"] = multi_env(ncomm, world)
    except Exception as e:  # noqa: BLE001
        extra["multi_env"] = {"error": repr(e)}
    if ncomm is not None:
        from feddct_amd import comm as Cm
        from feddct_amd.comm import (FA_XCHG_RS_GATHER, NativeAggregator,
                                     NativeBlockedAggregator, NativeChainedAggregator,
                                     NativeShardedAggregator, NativeStripedAggregator,
                                     multi_select)
        # the DEFAULT entry first (r06: the exact form and chunk count the
        # cost model picks for these counts on this layout, result on the
        # last rank — the model's root; the form is in the name)
        form, fk, fus = multi_select(counts, layout=layout, detail=True)
        droot = last
        extra["default_choice"] = {"form": form, "nchunks": fk, "model_us": round(fus, 1)}
        run_mode(f"default={form}/native", lambda o32, o64: NativeAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, final="reduce", root=droot).step,
            droot, True, model=(Cm.MODE_IDS[form], fk))
        run_mode("blocked/native", lambda o32, o64: NativeBlockedAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, final="reduce", root=0).step, 0, True,
            model=(Cm.FA_MODE_BLOCKED, 1))
        run_mode("blocked/native/allreduce", lambda o32, o64: NativeBlockedAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, final="allreduce").step, -1, True,
            steps=max(5, args.steps // 2), model=(Cm.FA_MODE_BLOCKED, 1))
        # the chained round's chunk count and the striped round's, swept
        # (the model picks them; the first multi-GPU run checks it)
        for k in (4, 8, 16, 32):
            run_mode(f"chained/native/c{k}", lambda o32, o64, k=k: NativeChainedAggregator(
                layout, l32, l64, n_total, o32, o64, ncomm, nchunks=k, final="reduce",
                root=last).step, last, True, steps=max(5, args.steps // 4),
                model=(Cm.FA_MODE_CHAINED, k))
        run_mode("chained/native/allreduce", lambda o32, o64: NativeChainedAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, nchunks=args.chain_chunks,
            final="allreduce").step, -1, True, steps=max(5, args.steps // 2),
            model=(Cm.FA_MODE_CHAINED, args.chain_chunks))
        run_mode("e1/native/reduce", lambda o32, o64: NativeShardedAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, nchunks=args.chunks,
            final="reduce").step, 0, False)
        run_mode("e1/native/rs_gather", lambda o32, o64: NativeShardedAggregator(
            layout, l32, l64, n_total, o32, o64, ncomm, nchunks=args.chunks, final="reduce",
            exchange=FA_XCHG_RS_GATHER).step, 0, False)
        if not args.no_exact:
            for k in (1, 2, 4, 8):
                run_mode(f"striped/native/c{k}", lambda o32, o64, k=k: NativeStripedAggregator(
                    layout, l32, l64, n_total, o32, o64, ncomm, final="reduce", root=last,
                    nchunks=k).step, last, True, steps=max(5, args.steps // 4),
                    model=(Cm.FA_MODE_STRIPED, k))
    run_mode("chained/torch.distributed", lambda o32, o64: (lambda a: lambda: a.step(l32, l64))(
        ChainAggregator(layout, n_total, o32, o64, group=group, final="reduce", root=last,
                        nchunks=args.chain_chunks)), last, True, steps=max(5, args.steps // 2))
    run_mode("e1/torch.distributed", lambda o32, o64: ShardedAggregator(
        layout, l32, l64, n_total, o32, o64, nchunks=args.chunks, final="reduce").step, 0, False)
    run_mode("e1/torch.distributed/rs_gather", lambda o32, o64: ShardedAggregator(
        layout, l32, l64, n_total, o32, o64, nchunks=args.chunks, final="reduce",
        exchange="rs_gather").step, 0, False)
    striped_host = None
    if not args.no_exact and not args.kernel_only:
        try:
            with phase("e2/torch.distributed"):
                striped, striped_host, hbufs = exact_modes(
                    layout, manifest, clients, out32, out64, world, group, dev, nbytes_rank,
                    max(3, min(5, args.steps // 10)))
            modes["e2/torch.distributed"] = {"t": striped["ms_per_step"] / 1e3, "root": 0,
                                             "out": hbufs[0:2], "exact_class": True}
        except Exception as e:  # noqa: BLE001
            modes["e2/torch.distributed"] = {"error": repr(e)}
    # parity of every mode on rank 0 (results on another rank travel there)
    with phase("parity"):
        ex32 = ex64 = None
        if rank == 0:
            allc = make_clients(layout, manifest, range(n_total), dev)
            ex32, ex64 = torch.zeros_like(out32), torch.zeros_like(out64)
            Reducer(layout, allc, ex32, ex64)()
            torch.cuda.synchronize()
            del allc
        segmask = torch.zeros(out32.numel(), dtype=torch.bool, device=dev)
        for o, m in layout.segs32:
            segmask[int(o):int(o + m)] = True
        report = {}
        for name in sorted(modes):
            m = modes[name]
            if "error" in m:
                report[name] = {"error": m["error"]}
                continue
            o32, o64 = m["out"]
            src = 0 if m["root"] < 0 else m["root"]
            if src != 0:
                from feddct_amd.dist import p2p
                if rank == src:
                    p2p([(dist.isend, o32, 0), (dist.isend, o64, 0)], group)
                elif rank == 0:
                    p2p([(dist.irecv, o32, src), (dist.irecv, o64, src)], group)
            r = {"ms_per_step": round(m["t"] * 1e3, 4),
                 "GBps": round(nbytes_rank * world / m["t"] / 1e9, 2),
                 "result_on": "every rank" if m["root"] < 0 else f"rank {m['root']}"}
            for k in ("model_us", "profile"):
                if k in m:
                    r[k] = m[k]
            if rank == 0:
                # every element of every key (the padding between keys is no
                # tensor's and each mode leaves it as it likes)
                a32, b32 = o32[segmask].view(torch.int32), ex32[segmask].view(torch.int32)
                same = bool(torch.equal(a32, b32) and torch.equal(o64, ex64))
                r["bit_exact"] = same
                if not same:
                    r["max_ulp_fp32"] = ulp_dist(o32[segmask], ex32[segmask])
                    r["ulp_histogram_fp32"] = ulp_hist(o32[segmask], ex32[segmask])
                    r["int64_bit_exact"] = bool(torch.equal(o64, ex64))
            report[name] = r
        # the headline: the fastest EXACT-class mode whose result is the
        # reference's bits (an e1 round is bit-exact by accident at one rank:
        # never the headline) — decided on rank 0, shared so every rank agrees
        best_t, best = float("inf"), ""
        if rank == 0:
            for name, r in report.items():
                if (r.get("bit_exact") and modes[name]["exact_class"]
                        and modes[name]["t"] < best_t):
                    best_t, best = modes[name]["t"], name
        sel = [best, best_t]
        dist.broadcast_object_list(sel, src=0, group=group)
        best, best_t = sel
    if not best:   # no exact mode ran: report the exact class's fastest, flagged
        cands = [n for n, m in modes.items() if "t" in m and m["exact_class"]]
        best = min(cands, key=lambda n: modes[n]["t"]) if cands else min(
            (n for n in modes if "t" in modes[n]), key=lambda n: modes[n]["t"])
        best_t = modes[best]["t"]
        extra["headline_not_verified_exact"] = True
    extra["modes"] = report
    extra["selected_mode"] = best
    mc = model_check(report)
    if mc:
        extra["model_check"] = mc
    # the opt-in re-associated round beside the exact headline: its time and
    # its distance from the reference's bits
    e1 = [n for n in report if n.startswith("e1/") and "ms_per_step" in report[n]]
    if e1:
        f = min(e1, key=lambda n: report[n]["ms_per_step"])
        extra["e1_reassociated_opt_in"] = {
            "mode": f, "ms_per_step": report[f]["ms_per_step"],
            "bit_exact": report[f].get("bit_exact"),
            "max_ulp_fp32": report[f].get("max_ulp_fp32"),
            "note": "not the default; NOT within north_star's 1 ULP"}
    if striped_host is not None:
        extra["exact_mode_host_ingress"] = striped_host
    if not args.kernel_only:
        log(f"[rank {rank}] config 5 sharded")
        try:
            with phase("config 5 sharded"):
                extra["cfg5_feddct_c100_n24_sharded"] = cfg5_sharded(
                    dev, world, rank, group, max(10, args.steps // 2), ncomm, args.chain_chunks)
        except Exception as e:  # noqa: BLE001
            extra["cfg5_feddct_c100_n24_sharded"] = {"error": repr(e)}
    return best_t, t_kernel, ncomm

def model_check(report):
    """The cost model against the run: for every mode
    with a modelled time, measured / modelled; whether the model's fastest
    form is the measured fastest, and the measured time of the model's pick
    over the measured best (1.0: the model chose right).  None when fewer than
    two modes carry both numbers."""
    rows = {n: (r["ms_per_step"] * 1e3, r["model_us"]) for n, r in report.items()
            if "model_us" in r and "ms_per_step" in r and r["model_us"] > 0
            and not n.startswith("default=")}
    if len(rows) < 2:
        return None
    ratio = {n: round(t / m, 3) for n, (t, m) in rows.items()}
    pick = min(rows, key=lambda n: rows[n][1])
    best = min(rows, key=lambda n: rows[n][0])
    return {"measured_over_model": ratio, "model_pick": pick, "measured_best": best,
            "agree": pick == best, "pick_over_best": round(rows[pick][0] / rows[best][0], 3)}


def multi_env(ncomm, world):
    """What the first real multi-GPU run needs to be read (VERDICT r05 next
    4): the RCCL / NCCL / HSA / HIP environment of this process, the
    communicator's rank count as RCCL reports it, and which devices this
    process sees can access each other's memory (hipDeviceCanAccessPeer)."""
    from feddct_amd import comm as Cm
    env = {k: v for k, v in sorted(os.environ.items())
           if k.startswith(("RCCL_", "NCCL_", "HSA_", "HIP_", "GPU_MAX_HW_QUEUES"))}
    # no native communicator (a gloo rehearsal, --same-device): the rest only
    n, r, d = ncomm.info() if ncomm is not None else (None, None, None)
    ndev = torch.cuda.device_count()
    peer = [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(ndev)]
            for i in range(ndev)]
    return {"env": env, "comm_count": n, "comm_rank": r, "comm_device": d, "world": world,
            "visible_devices": ndev, "peer_access": peer,
            # in effect in this process (FA_MODEL_* environment overrides)
            "model_constants": Cm.model_constants()}


def build_line(args, world, nbytes_rank, bytes_per_client, t_step, t_kernel, extra):
    """The one JSON line (bench contract) from the measured times + extras."""
    achieved = nbytes_rank / t_kernel / 1e9
    traffic, traffic_src = pmc_traffic(world)
    line = {
        "metric": METRIC,
        "value": round(nbytes_rank * world / t_step / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (portable integer-hash PRNG, feddct_amd/synth.py; seeds 1000+client)",
        "config": {"workload": f"FedAvg {N_CLIENTS} clients/GPU x wide_resnet16_8 CIFAR-10 "
                               "(82 fp32 + 16 int64 keys), unweighted mean (reference semantics)",
                   "clients_per_gpu": N_CLIENTS, "bytes_per_client": bytes_per_client,
                   "algorithmic_bytes_per_step": nbytes_rank * world,
                   "parallelism": (f"client shards x{world}: {extra.get('selected_mode')} "
                                   "(fastest bit-exact round form; all forms in 'modes')"
                                   if extra.get("selected_mode") else "single GPU")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_pmc": traffic_src,
                     "kernel_us": round(t_kernel * 1e6, 2)},
        "cpu_baseline": None,
        "host": os.uname().nodename,
    }
    try:
        line["gpu"] = torch.cuda.get_device_name(0)
    except Exception:  # noqa: BLE001  (CPU-only helper tests)
        line["gpu"] = None
    line.update(extra)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--chunks", type=int, default=8)
    ap.add_argument("--chain-chunks", type=int, default=16,
                    help="N>1: column chunks of the chained round's state hops")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact", action="store_true",
                    help="N>1: skip timing the column-striped exact mode")
    ap.add_argument("--cpu-budget", type=float, default=25.0)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse ranks on one GPU")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--kernel-only", action="store_true",
                    help="only the timed reduce launches (for rocprofv3 runs)")
    ap.add_argument("--multi-rehearsal", action="store_true",
                    help="run the N>1 path (every round form, native RCCL communicator "
                         "included) with however many ranks there are, also one: a "
                         "one-GPU rehearsal of the driver's multi-GPU command")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    multi = world > 1 or args.multi_rehearsal
    if multi:
        # diagnosis only: a multi-rank run that stalls leaves every rank's
        # Python stack on stderr (nothing is interrupted)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ.get("FA_BENCH_STACK_DUMP_S", "480")))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if args.same_device:
        local_rank = 0
    idle_state = None
    if world == 1 and not args.kernel_only:
        try:
            idle_state = gpu_state_idle()
        except Exception as e:  # noqa: BLE001  (reported, never fatal)
            idle_state = {"error": repr(e)}
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    group = None
    if multi:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        group = dist.group.WORLD

    manifest = load_manifest(LAYOUT)
    layout = BucketLayout.from_manifest(manifest)
    first = rank * N_CLIENTS
    clients = make_clients(layout, manifest, range(first, first + N_CLIENTS), dev)
    # the global's bucket from the same slab as the clients' (slab.py), as the
    # drop-in's arenas place them
    out32 = slab.carve(clients[0][0].numel(), torch.float32, dev)
    out64 = torch.zeros_like(clients[0][1])
    reducer = Reducer(layout, clients, out32, out64)
    nbytes_rank = layout.algorithmic_bytes(N_CLIENTS)
    torch.cuda.synchronize()

    extra = {}
    if idle_state is not None:
        extra["gpu_state_idle"] = idle_state
    ncomm = None
    if not multi:
        per = []
        if not args.kernel_only:
            # streaming work BEFORE the headline's own W warmups, so the
            # timed steps do not see the clocks ramp: the copy ceiling of this
            # box, the weighted and broadcast variants of the same reduction
            # non-zero data on both sides: zero-filled buffers stream faster on
            # this chip than real data (tools/bcastlab.hip: the same broadcast
            # 130 us on zeros, 169 us on hashed values), which would overstate
            # the ceiling
            big = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)  # 1 GiB
            big.uniform_(-1.0, 1.0)
            big2 = torch.empty_like(big).uniform_(-1.0, 1.0)

            def copy_big():
                _lib.check(_lib.lib.fa_copy_f32(big.data_ptr(), big2.data_ptr(), big.numel(),
                                                torch.cuda.current_stream().cuda_stream))
            tc, _ = timed_launches(copy_big, 100, 3)   # ~33 ms of streaming
            extra["copy_ceiling_GBps"] = round(2 * big.numel() * 4 / tc / 1e9, 1)
            # and its read-only ceiling (the reduce is 95 % reads): the same
            # 1 GiB read in the reduce's own tile shape, nothing stored
            sink = torch.zeros(256, dtype=torch.float32, device=dev)

            def read_big():
                _lib.check(_lib.lib.fa_read_probe_f32(big.data_ptr(), big.numel(),
                                                      sink.data_ptr(), 0,
                                                      torch.cuda.current_stream().cuda_stream))
            # best of three passes of 30 (~4 ms each)
            tr = min(timed_launches(read_big, 30, 3)[0] for _ in range(3))
            extra["read_ceiling_GBps"] = round(big.numel() * 4 / tr / 1e9, 1)
            del big, big2, sink
            # weighted variant (client-size weights, BASELINE config 4's extension)
            from feddct_amd.aggregate import client_weights as weights_from_sizes
            w = weights_from_sizes(np.arange(1, N_CLIENTS + 1))
            wo32, wo64 = torch.zeros_like(out32), torch.zeros_like(out64)
            wred = Reducer(layout, clients, wo32, wo64, weights=w, plan=reducer.plan)
            wper = []
            tw, _ = timed_launches(wred, max(100, args.steps // 2), max(20, args.warmup))
            extra["weighted_GBps"] = round(nbytes_rank / tw / 1e9, 1)
            extra["weighted_us"] = round(tw * 1e6, 2)
        # the headline straight after the streaming above: no host-side check
        # (digest hashing idles the GPU for ~0.1 s) between them and its W
        # warm-ups
        t_step, wall = timed_launches(reducer, args.steps, args.warmup)
        t_kernel = t_step
        if "read_ceiling_GBps" in extra:
            # this box's own bound: the headline as a fraction of the copy and
            # of the read-only rate measured just before it
            gbs = nbytes_rank / t_step / 1e9
            extra["headline_vs_box_ceilings"] = {
                "copy": round(gbs / extra["copy_ceiling_GBps"], 4),
                "read_only": round(gbs / extra["read_ceiling_GBps"], 4)}
        if not args.kernel_only:
            timed_launches(wred, max(100, args.steps // 2), 20, per_launch=wper)
            extra["weighted_launch"] = launch_stats(wper)
            extra["weighted_parity"] = weighted_digest_check("wrn16_8_c10/n20/sizes_1_20",
                                                             layout, wo32, wo64)
            del wred, wo32, wo64
            # the same launches once more with an event between consecutive
            # launches (kept out of the headline's timed region: the extra
            # event packets add a few µs between kernels) — the spread and
            # any clock ramp across K launches
            timed_launches(reducer, args.steps, 20, per_launch=per)
            extra["headline_launch"] = launch_stats(per)
            extra["slab_vs_separate_allocations"] = separate_allocations_ab(
                layout, clients, reducer, out32, out64)
            try:
                extra["gpu_state"] = gpu_state_under_load(reducer)
            except Exception as e:  # noqa: BLE001  (reported, never fatal)
                extra["gpu_state"] = {"error": repr(e)}
            with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
                want = json.load(f)[f"fedavg/{LAYOUT}/n{N_CLIENTS}"]
            got = digest_of(layout, out32, out64)
            extra["parity"] = {"vs": "reference server_aggregate SHA-256 (tests/golden)",
                               "bit_exact": got == want}
            extra["host_inclusive"] = host_inclusive(layout, clients, reducer, out32, out64)
            try:
                extra["torch_gpu_order_mode"] = torch_gpu_order_mode(layout, clients)
            except Exception as e:  # noqa: BLE001
                extra["torch_gpu_order_mode"] = {"error": repr(e)}
            # the same at N = 32, where torch splits the large tensors' rows
            # in two (S = 2), beside the default order's time
            try:
                more = make_clients(layout, manifest, range(first + N_CLIENTS, first + 32), dev)
                c32 = clients + more
                m32 = torch_gpu_order_mode(layout, c32)
                d32, d64 = torch.zeros_like(out32), torch.zeros_like(out64)
                td, _ = timed_launches(Reducer(layout, c32, d32, d64), 20, 3)
                m32["default_order_us"] = round(td * 1e6, 1)
                m32["n"] = 32
                extra["torch_gpu_order_mode_n32"] = m32
                del more, c32, d32, d64
                torch.cuda.empty_cache()
            except Exception as e:  # noqa: BLE001
                extra["torch_gpu_order_mode_n32"] = {"error": repr(e)}
            # the round with its broadcast (FA_F_BCAST: reduce launch + broadcast
            # launch over the same tiles), N*B read + (N+1)*B written — after
            # every measurement that needs the clients' own values
            extra["round"] = round_block(layout, clients, out32, out64, reducer.plan,
                                         extra, max(20, args.steps // 2))
            extra["round_with_broadcast_us"] = extra["round"]["us"]
            # the write probe overwrote the client buckets: their synthetic
            # state again, for the drop-in timings and the CPU baseline below
            # 
            from feddct_amd.workload import fill_client
            for j, (c32, c64) in enumerate(clients):
                fill_client(layout, manifest, c32, c64, first + j)
            torch.cuda.synchronize()
            extra["dropin"] = dropin_timing(layout, clients, dev)
            try:
                extra["dropin_feddct_cfg3"] = dropin_feddct_timing(dev)
            except Exception as e:  # noqa: BLE001
                extra["dropin_feddct_cfg3"] = {"error": repr(e)}
            try:
                extra["dropin_feddct_cfg5"] = dropin_feddct_timing(dev, n=24, classes=100)
            except Exception as e:  # noqa: BLE001
                extra["dropin_feddct_cfg5"] = {"error": repr(e)}
            extra["other_configs"] = other_configs(dev)
            try:
                extra["next_rows"] = next_rows(dev)
            except Exception as e:  # noqa: BLE001
                extra["next_rows"] = {"error": repr(e)}
            try:
                extra["cfg1_host_resident_n2"] = cfg1_host_resident(dev)
            except Exception as e:  # noqa: BLE001
                extra["cfg1_host_resident_n2"] = {"error": repr(e)}
    else:
        t_step, t_kernel, ncomm = multi_gpu(args, world, rank, dev, group, layout, manifest,
                                            clients, out32, out64, reducer, nbytes_rank, extra)

    line = build_line(args, world, nbytes_rank, layout.state_bytes(), t_step, t_kernel, extra)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.kernel_only:
        try:
            line["cpu_baseline"] = run_cpu_baseline(layout, manifest, clients, args.cpu_budget)
        except Exception as e:  # report, never hide
            line["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if multi:
        if ncomm is not None:
            ncomm.close()  # the library's communicator before torch's teardown
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
