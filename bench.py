#!/usr/bin/env python3
"""Benchmark: PCG + Jacobi iterations/s on the 5-point FDLaplacian2D, SpMV vs the HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--side M]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one PCG iteration (PCGSolver.py:109-138: SpMV, 2 dots + norm, 3 updates, Jacobi
apply) over the whole matrix. The headline workload is the metric's own (BASELINE.json: "5-pt
Laplacian N=10M"): A = FDLaplacian2D(-1, 1, 3163) (n = 10,004,569) generated on the device
(bit-identical to examples/FDLaplacian2D.py), b = A @ default_rng(12345).random(n),
control = CommonSolverArgs(maxiter=K, tau=0, failOnMaxiter=False) so exactly K iterations run
(PCGSolver.py:129-131). It is fixed for every N (strong scaling): with N > 1 the rows are split on
whole grid lines across ranks (one process per GPU), halo lines are exchanged with ncclSend/Recv
and the dot partials all-gathered with RCCL over xGMI, all inside libpsk. configs[3]'s 16384^2
system is timed the same way at the same N (`strong_scaling_16384`: the series the north star's
>= 6x 1 -> 8 GPU target is quoted on).

Timed region: barrier + device sync, ONE psk_pcg call of K iterations, device sync + barrier;
max over ranks; --repeats such regions, value = the median one. `roofline` prices the in-loop SpMV
(the metric's kernel) from HIP events recorded by libpsk on its own stream around every SpMV launch
of the median region; `traffic` comes from a rocprofv3 PMC profile of the SAME libpsk.so build
(sha256-checked) or is null. On rank 0 at N = 1 the extra keys time the general-matrix path,
configs[1] (4096^2), GMRES(30) Arnoldi steps (4096^2), configs[2] (GMRES(30)+ILUT, 2896^2),
configs[4] (PCG+AMG, 8192^2) and the CPU oracle at N = 10M (`cpu_baseline`).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "CG iterations/sec + SpMV GB/s vs HBM roofline, 5-pt Laplacian N=10M"
# libpsk times every EVENT_STRIDE-th SpMV launch of a timed region between two HIP events (an event
# pair around every launch cost ~5% of the iteration rate at N = 10M)
EVENT_STRIDE = 8
METRIC_SIDE = 3163              # FDLaplacian2D side of the metric's N = 10M: n = 10,004,569
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def fd_sizes(m):
    n = m * m
    nnz = 1 if m == 1 else 5 * n - 4 * m
    return n, nnz


def spmv_bytes(n, nnz):
    """Algorithmic SpMV bytes: vals+colidx, rowptr, x once, y written."""
    return 12 * nnz + 4 * (n + 1) + 16 * n


PCG_VEC_BYTES_PER_ROW = 73   # K2 (r, Ap, dinv in; r out) + K3 (r, p, dinv in; p out; x and p_{k-7..k-1} every 8th iteration), Jacobi
LAYOUT_NAMES = {0: "csr", 1: "sliced", 2: "sliced_wide", 3: "sliced_dict", 4: "diag"}   # PSK_LAYOUT_*


def pcg_iter_bytes(n, nnz, jacobi=True):
    """Compulsory bytes of one PCG iteration in libpsk's 3-launch schedule with a CSR SpMV
    (SURVEY.md §8d)."""
    return spmv_bytes(n, nnz) + (PCG_VEC_BYTES_PER_ROW if jacobi else 58) * n


def vec_bytes_per_row(N, M):
    """K2 + K3 bytes per row, averaged over iterations: K2 24 (r, Ap read, r written); K3 reads r and
    p_k and writes p_{k+1} every iteration, and x (read + write) with p_{k-7} .. p_{k-1} every 8th
    iteration only (the deferred x update, pcg.hip kPcgDefer) = 24 + 72/8; + 16 for a streamed
    DInv (K2 and K3 read it). 57 when the Jacobi diagonal is one scalar (psk_prec_jacobi_uniform),
    73 otherwise."""
    u = N.I32()
    N.check(N.lib.psk_prec_jacobi_uniform(M, ctypes.byref(u), None), "psk_prec_jacobi_uniform")
    return PCG_VEC_BYTES_PER_ROW - (16 if u.value else 0)


def layout_bytes(N, A, n):
    """Bytes one SpMV of A must move in its current storage layout — the matrix stream
    (psk_csr_layout) + x read once + y written — and the layout's name."""
    lay, stream = N.I32(), N.I64()
    N.check(N.lib.psk_csr_layout(A, -1, ctypes.byref(lay), None, None, ctypes.byref(stream)), "psk_csr_layout")
    return stream.value + 16 * n, LAYOUT_NAMES[lay.value]


class Liveness:
    """Progress that advances only when work completes, and a watchdog on it (round 6).

    `tick` is called when a libpsk call returns (bench wraps N.check), when a timed region or solve ends, and
    at host setup sub-steps; `phase` names what runs now and whether it is GPU work ("gpu": libpsk calls
    return every few seconds at most) or one long host call ("host": SuperLU's spilu at 2896^2, the SA setup,
    the CPU oracle). A daemon thread prints, every `beat_s`, the phase, the progress counter and the age of its
    last advance; when the counter has not advanced for the phase's limit it prints the stuck phase and ends
    the process with exit code 3 (no restart, no re-exec) instead of leaving a stalled device call to the
    driver's time limit. The printed line changes only with the counter and its age, so a stall reads as one."""

    def __init__(self, gpu_stall_s=150.0, host_stall_s=420.0, beat_s=30.0, clock=time.monotonic, write=None,
                 exit_fn=None):
        self.gpu_stall_s, self.host_stall_s, self.beat_s = gpu_stall_s, host_stall_s, beat_s
        self.clock = clock
        self.write = write or (lambda msg: (sys.stderr.write(msg + "\n"), sys.stderr.flush()))
        self.exit_fn = exit_fn or os._exit
        self.t_start = clock()
        self.name, self.kind, self.count, self.what = "start", "host", 0, "start"
        self.t_last = self.t_phase = self.t_start

    def phase(self, name, kind="gpu"):
        self.name, self.kind = name, kind
        self.t_phase = self.clock()
        self.tick("phase " + name)
        self.write("bench: %s (%s phase, t=%.1f s)" % (name, kind, self.t_phase - self.t_start))

    def tick(self, what=""):
        self.count += 1
        self.what = what
        self.t_last = self.clock()

    def limit(self):
        return self.gpu_stall_s if self.kind == "gpu" else self.host_stall_s

    def line(self):
        now = self.clock()
        return "bench: %s [%s] progress %d, last: %s %.0f s ago (phase %.0f s)" % (
            self.name, self.kind, self.count, self.what, now - self.t_last, now - self.t_phase)

    def stalled(self):
        """The watchdog's verdict now: None, or the message it ends the run with."""
        age = self.clock() - self.t_last
        if age <= self.limit():
            return None
        return ("bench: WATCHDOG: no progress in %s phase '%s' for %.0f s (limit %.0f s; last advance: %s, "
                "progress %d): exiting with code 3" % (self.kind, self.name, age, self.limit(), self.what, self.count))

    def start(self):
        import threading

        def run():
            while True:
                time.sleep(self.beat_s)
                self.write(self.line())
                msg = self.stalled()
                if msg:
                    self.write(msg)
                    self.exit_fn(3)
                    return
        threading.Thread(target=run, daemon=True).start()


LIVE = Liveness()


def progress(name, kind="gpu"):
    """Phase marker on stderr (stdout carries only the JSON line), with the watchdog's phase kind."""
    LIVE.phase(name, kind)


def _watch_libpsk(N):
    """Every libpsk call that returns through N.check (bench's own calls and the pysolvers_amd classes') is a
    progress tick: a kernel that never finishes blocks inside its call and stops the counter."""
    check = N.check

    def checked(rc, where):
        LIVE.tick(where)
        return check(rc, where)
    N.check = checked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--side", type=int, default=METRIC_SIDE,
                    help="grid side m of FDLaplacian2D for the headline (n = m^2 rows; 3163 = the metric's N=10M)")
    ap.add_argument("--scaling-side", type=int, default=16384,
                    help="also time configs[3]'s 16384^2 system at this N (the strong-scaling series; 0 = skip)")
    ap.add_argument("--scaling-steps", type=int, default=50)
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed regions of --steps iterations each; value = the median (SURVEY.md §8d)")
    ap.add_argument("--cpu-iters", type=int, default=50, help="timed oracle iterations for cpu_baseline (0 = skip)")
    ap.add_argument("--general", type=int, default=1,
                    help="also time the general-matrix path (double values, streamed DInv) on rank 0")
    ap.add_argument("--config2", type=int, default=1, help="also time configs[2] (GMRES(30)+ILUT, FD 2896^2) on rank 0")
    ap.add_argument("--config4", type=int, default=1, help="also time configs[4] (PCG+AMG, -FD 8192^2) on rank 0")
    ap.add_argument("--config1", type=int, default=1, help="also time configs[1] (PCG+Jacobi 4096^2) on rank 0")
    ap.add_argument("--gmres", type=int, default=1, help="also time GMRES(30)+Jacobi Arnoldi steps at 4096^2 on rank 0")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r6_pmc_traffic_%d.json"),
                    help="PMC traffic summary (tools/pmc_summary.py) of the same build; %%d = the side")
    args = ap.parse_args()
    LIVE.write("bench: start (pid %d, python %s)" % (os.getpid(), sys.version.split()[0]))

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched as `python bench.py --gpus N` (no torchrun): start the N ranks ourselves. Nothing in
        # this process has touched the GPU (libpsk is imported by the ranks only).
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    maps_out = os.environ.get("PSK_DUMP_MAPS")
    if maps_out:
        # registered before libpsk's own atexit hook, so it runs after it (LIFO): the process's
        # mappings as exit() starts tearing libraries down, to resolve a fault PC to library + offset
        import atexit
        atexit.register(_dump_maps, maps_out)

    # One rank never imports torch (torch.distributed is the N > 1 control plane only): libpsk then runs on
    # the system ROCm runtime alone. With torch's bundled HIP runtime in the process, a rocprofv3 run
    # faulted in exit(): the profiler's HSA (loaded first) served torch's HIP, and torch's HIP teardown
    # called into it after the profiler had finalised it (profiles/r4_exit_fault.txt).
    if world == 1:
        os.environ.setdefault("PSK_NO_TORCH", "1")
    LIVE.start()   # from here a stall of more than the phase's limit ends the run (exit 3) with its phase named
    progress("start-up: load libpsk (HIP runtime)", "host")
    from pysolvers_amd import _native as N
    _watch_libpsk(N)
    progress("start-up: device selection")
    # one GPU per rank: LOCAL_RANK when every GPU is visible to every rank; a launcher that narrows
    # visibility per rank leaves one device (ordinal 0) per process
    ndev = N.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    dev = int(os.environ.get("PSK_BENCH_DEVICE", local_rank if local_rank < ndev else local_rank % ndev))
    N.check(N.lib.psk_set_device(dev), "psk_set_device")

    dist = None
    if world > 1:
        progress("start-up: torch.distributed (gloo control plane)", "host")
        import torch.distributed as dist
        # control plane only. Gloo's C++ connection log goes to fd 1; keep stdout for the ONE JSON
        # line the driver parses by pointing fd 1 at stderr while the group connects
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    def barrier():
        if dist is not None:
            dist.barrier()

    comm = ctypes.c_void_p()
    # PSK_BENCH_TRANSPORT=host: rehearsal of the N>1 path with all ranks on ONE GPU (collectives over
    # host shared memory, psk_comm_init_host); never a measurement
    transport = os.environ.get("PSK_BENCH_TRANSPORT", "rccl")
    if world > 1 and transport == "host":
        obj = [("/psk_bench_%d_%s" % (os.getpid(), os.urandom(6).hex())).encode() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        N.check(N.lib.psk_comm_init_host(world, rank, obj[0], ctypes.byref(comm)), "psk_comm_init_host")
    elif world > 1:
        uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES)()
        if rank == 0:
            N.check(N.lib.psk_comm_unique_id(uid), "psk_comm_unique_id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
        N.check(N.lib.psk_comm_init(world, rank, uid, ctypes.byref(comm)), "psk_comm_init")
    # the ranks' dot products: device-side stores into a host-shared mailbox (default; one node) or RCCL
    # all-gathers (PSK_DOT_TRANSPORT=rccl); the halo of p always goes over the transport above
    dots = os.environ.get("PSK_DOT_TRANSPORT", "mailbox")
    dots_note = None
    if world > 1 and dots == "mailbox":
        obj = [("/psk_mb_%d_%s" % (os.getpid(), os.urandom(6).hex())).encode() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        N.check(N.lib.psk_comm_mailbox(comm, obj[0]), "psk_comm_mailbox")
        # self-check (known values through the solvers' kernel stores and gather, bounded waits); every
        # rank's verdict is shared, so all fall back to RCCL all-gathers together when any rank failed
        rc = N.lib.psk_comm_mailbox_check(comm, 8)
        import torch
        flag = torch.tensor([0 if rc == 0 else 1], dtype=torch.int32)
        dist.all_reduce(flag)
        if int(flag.item()) != 0:
            dots_note = "mailbox self-check failed on %d rank(s): RCCL all-gathers used" % int(flag.item())
            N.lib.psk_comm_destroy(comm)
            comm = ctypes.c_void_p()
            if transport == "host":
                obj = [("/psk_bench_%d_%s" % (os.getpid(), os.urandom(6).hex())).encode() if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                N.check(N.lib.psk_comm_init_host(world, rank, obj[0], ctypes.byref(comm)), "psk_comm_init_host")
            else:
                uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES)()
                if rank == 0:
                    N.check(N.lib.psk_comm_unique_id(uid), "psk_comm_unique_id")
                obj = [bytes(uid)]
                dist.broadcast_object_list(obj, src=0)
                uid = (ctypes.c_uint8 * N.PSK_UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
                N.check(N.lib.psk_comm_init(world, rank, uid, ctypes.byref(comm)), "psk_comm_init")
            dots = "rccl"

    # ---- the headline: the metric's N = 10M system on `world` GPUs ----------------------------------
    progress("headline N=%d" % (args.side * args.side))
    m = args.side
    n, nnz = fd_sizes(m)
    sys_ = PcgSystem(N, m, comm if world > 1 else None, world)
    regions = sys_.regions(args.steps, args.warmup, args.repeats, barrier, dist)
    imed = sorted(range(len(regions)), key=lambda i: regions[i][0])[len(regions) // 2]
    dt, spmv_ms_med, spmv_launches = regions[imed]

    out = None
    if rank == 0:
        it_s = args.steps / dt
        nloc_r0 = sys_.nloc
        bspmv = spmv_bytes(nloc_r0, sys_.nnz_loc)
        blay, lname, lay = sys_.layout()
        # the bytes this launch must move in its storage layout (matrix stream + x read + y written;
        # DESIGN.md §5); with a value dictionary far fewer than CSR's 12 B/entry
        ach = blay / (spmv_ms_med * 1e-3) / 1e9 if spmv_ms_med > 0 else None
        csr_eq = bspmv / (spmv_ms_med * 1e-3) / 1e9 if spmv_ms_med > 0 else None
        vb = vec_bytes_per_row(N, sys_.M)
        biter = blay * world + vb * n
        pmc = pmc_traffic(args.traffic_json % m, m, world, mode=1, sliced=lay != N.PSK_LAYOUT_CSR)
        out = {
            "metric": METRIC,
            "value": it_s,
            "unit": "CG iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"iters": sys_.settle_iters(), "note": "one untimed solve (~0.3 s; same count on every rank) after "
                                                             "the warm-up iterations, right before the first timed region"},
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: FDLaplacian2D(-1,1,m) built on device (bit-identical to the reference "
                    "generator), b = A @ default_rng(12345).random(n)",
            "config": {"workload": "PCG+Jacobi, FDLaplacian2D %dx%d (n=%d, nnz=%d; the metric's N=10M), tau=0 "
                                   "fixed-iteration" % (m, m, n, nnz),
                       "m": m, "precond": "jacobi", "parallelism": "row-block x%d (%s)" % (world, "RCCL" if transport == "rccl" else "host-shm rehearsal")
                       if world > 1 else "single GPU",
                       "transport": {"halo": "rccl send/recv" if transport == "rccl" else "host-shm rehearsal",
                                     "dots": "mailbox (kernel stores to host-shared memory)" if dots == "mailbox"
                                     else ("rccl allgather" if transport == "rccl" else "host-shm allgather"),
                                     "dots_note": dots_note}
                       if world > 1 else None},
            "repeats": {"regions": len(regions), "value_is": "median region",
                        "it_s": [args.steps / r[0] for r in regions],
                        "spmv_avg_launch_ms": [r[1] for r in regions]},
            "roofline": {"bound": "hbm", "kernel": pmc.pop("kernel", None) or spmv_kernel_label(lay, 1),
                         "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": (ach / HBM_PEAK_GBPS) if ach else None,
                         **pmc,
                         "algorithmic_bytes_per_launch": blay, "avg_launch_ms": spmv_ms_med,
                         "launches": spmv_launches, "layout": lname,
                         "timing": "HIP events libpsk records on its own stream around every %d-th SpMV launch (iteration 0's runs inside the fused init launch on the diagonal layout) "
                                   "of the median timed region (rank 0's events; max over ranks at N > 1)" % EVENT_STRIDE,
                         "csr_bytes_per_launch": bspmv,
                         "csr_count_over_time_GBps": csr_eq,
                         "csr_count_note": "SURVEY §8d's CSR byte count (12 nnz + 4(n+1) + 16n) over the same time: "
                                           "NOT a bandwidth — the layout streams fewer bytes than CSR",
                         "bound_note": ("diag layout, 17 B/row: the launch is bound by one memory round trip per "
                                        "wave (latency) and its dot epilogue, not by HBM bandwidth; "
                                        "pcg_iteration_roofline prices the whole iteration (DESIGN.md §4)")
                         if lname == "diag" else None},
            "pcg_iteration_roofline": {"bytes_per_iteration": biter, "vector_bytes_per_row": vb,
                                       "achieved_GBps": biter * it_s / 1e9,
                                       "frac_of_aggregate_peak": biter * it_s / 1e9 / (HBM_PEAK_GBPS * world)},
            "setup_s": sys_.setup_s,
        }
        if world == 1:
            # what the sampled per-launch HIP events of the timed regions cost: the same regions without them
            ne = sys_.regions(args.steps, 0, 3, barrier, dist, events=False)
            out["regions_without_kernel_events"] = {"it_s": [args.steps / r[0] for r in ne],
                                                    "median_it_s": args.steps / median([r[0] for r in ne])}
            # the same matrix, plain y = A x launches back to back (no dot epilogue, no solver kernels
            # in between): how much of the in-loop SpMV time is the PCG context
            bms = ctypes.c_double()
            N.check(N.lib.psk_spmv_timed(sys_.A, sys_.db, sys_.dsol, 50, ctypes.byref(bms)), "psk_spmv_timed")
            pbb = pmc_traffic(args.traffic_json % m, m, 1, mode=0, sliced=lay != N.PSK_LAYOUT_CSR)
            out["spmv_plain_batch50"] = {"avg_launch_ms": bms.value,
                                         "achieved_GBps": blay / (bms.value * 1e-3) / 1e9,
                                         "frac": blay / (bms.value * 1e-3) / 1e9 / HBM_PEAK_GBPS, **pbb}
            progress("fixed_overhead")
            out["fixed_overhead"] = fixed_overhead(sys_, args.steps)
            if args.general:
                progress("general_path")
                out["general_path"] = general_path(N, sys_.A, sys_.db, sys_.dsol, m, args.steps)
            out["spmv_csr_layout_batch50"] = csr_layout_batch(N, sys_.A, sys_.db, sys_.dsol, bspmv, reps=50)
            # the north star's "CSR SpMV" inside the PCG loop: the same solve with the CSR layout
            out["csr_layout_in_loop"] = csr_in_loop(sys_, bspmv, args.steps)
        if world > 1:
            out["comm"] = comm_breakdown(sys_.comm[imed], dt / args.steps, spmv_ms_med, world)
        if transport == "host" and world > 1:
            out["rehearsal"] = "PSK_BENCH_TRANSPORT=host: all ranks on one GPU, host shared-memory collectives; not a measurement"
    sys_.free()

    # ---- configs[3]'s 16384^2 system at the same N: the strong-scaling series of the >= 6x target ----
    if args.scaling_side and args.scaling_side != m:
        ms_ = args.scaling_side
        progress("strong_scaling_%d" % ms_)
        big = PcgSystem(N, ms_, comm if world > 1 else None, world)
        reg = big.regions(args.scaling_steps, 5, 3, barrier, dist)
        if rank == 0:
            imb = sorted(range(len(reg)), key=lambda i: reg[i][0])[len(reg) // 2]
            dtb, smsb, _ = reg[imb]
            bl, lname, lay = big.layout()
            pm = pmc_traffic(args.traffic_json % ms_, ms_, world, mode=1, sliced=lay != N.PSK_LAYOUT_CSR)
            nb_, _ = fd_sizes(ms_)
            vbb = vec_bytes_per_row(N, big.M)
            out["strong_scaling_%d" % ms_] = {
                "workload": "PCG+Jacobi, FDLaplacian2D %dx%d (configs[3]), tau=0, %d iterations per region, "
                            "median of %d regions, same N as the headline" % (ms_, ms_, args.scaling_steps, len(reg)),
                "n_gpus": world, "pcg_it_per_s": args.scaling_steps / dtb, "ms_per_step": dtb * 1e3 / args.scaling_steps,
                "regions_it_s": [args.scaling_steps / r[0] for r in reg],
                "spmv_avg_launch_ms": smsb, "spmv_algorithmic_bytes_per_launch": bl, "layout": lname,
                "spmv_frac": bl / (smsb * 1e-3) / 1e9 / HBM_PEAK_GBPS, **pm,
                "pcg_iteration_frac_of_aggregate_peak":
                    (bl * world + vbb * nb_) * args.scaling_steps / dtb / 1e9 / (HBM_PEAK_GBPS * world)}
            if world > 1:
                out["strong_scaling_%d" % ms_]["comm"] = comm_breakdown(big.comm[imb], dtb / args.scaling_steps, smsb,
                                                                        world)
        big.free()

    if rank == 0:
        if world == 1 and args.config1 and m != 4096:
            progress("configs1_pcg_jacobi_4096")
            out["configs1_pcg_jacobi_4096"] = pcg_4096(N)
        if world == 1 and args.gmres:
            progress("gmres30_jacobi_4096")
            out["gmres30_jacobi_4096"] = gmres_arnoldi(N)
        if world == 1 and args.config2:
            progress("configs2_gmres30_ilut (host SuperLU ILUT first)", "host")
            out["configs2_gmres30_ilut"] = gmres_ilut(N)
        if world == 1 and args.config4:
            progress("configs4_pcg_amg_8192 (host SA setup first)", "host")
            out["configs4_pcg_amg_8192"] = pcg_amg(N)
        if world == 1 and args.cpu_iters > 0:
            progress("cpu_baseline", "host")
            out["cpu_baseline"] = cpu_baseline(m, args.cpu_iters)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)

    if world > 1:
        barrier()
        N.lib.psk_comm_destroy(comm)
        dist.destroy_process_group()


def comm_breakdown(comm, t_iter_s, spmv_ms, world):
    """The N > 1 line's own explanation of its iteration time: libpsk times, at the sampled
    iterations (every EVENT_STRIDE-th), this rank's p.Ap scalar gather (the mailbox gather kernel, whose duration
    is the wait for the slowest rank plus the transport; or the RCCL all-gather) and the halo exchange of p
    (pack + send/recv on the stream that runs it: the second stream when it overlaps K3); each is the max over
    ranks of the per-rank means. PCG has two such gathers per iteration (p.Ap after the SpMV, (r.r, u.r) after
    K2, the same shape), so the exposed-communication estimate is 2 x gather, plus the halo when it does not
    overlap K3 (PSK_HALO_OVERLAP=0)."""
    gat, halo, samples = comm
    overlap = os.environ.get("PSK_HALO_OVERLAP", "1") != "0"
    exposed = 2 * gat + (0.0 if overlap else halo)
    return {"ranks": world, "samples_per_rank": samples, "iteration_us": t_iter_s * 1e6,
            "spmv_us_max_rank": spmv_ms * 1e3, "gather_us_max_rank": gat * 1e3, "halo_us_max_rank": halo * 1e3,
            "halo_overlapped_with_K3": overlap, "exposed_comm_est_us": exposed * 1e3,
            "exposed_comm_share_of_iteration": exposed * 1e-3 / t_iter_s if t_iter_s > 0 else None,
            "timing": "HIP events libpsk records on every %d-th iteration of the median region (psk_result "
                      "gather_ms / halo_ms, ABI 4); max over ranks" % EVENT_STRIDE}


def _dump_maps(path):
    try:
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())
    except OSError:
        pass


def spawn_ranks(nranks):
    """One process per GPU without an external launcher: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
    for each child (rendezvous on 127.0.0.1), rank 0's JSON line forwarded to stdout, non-zero exit if
    any rank fails. The torchrun path (WORLD_SIZE already set) does not come here."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = procs[0].communicate()[0]
    codes = [p.wait() for p in procs]
    sys.stdout.write(out0.decode())
    sys.stdout.flush()
    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
    if bad:
        sys.stderr.write("bench.py: ranks failed (rank, exit code): %s\n" % bad)
        return 1
    return 0


def fixed_overhead(sys_, steps, short=20, reps=5):
    """The per-solve cost outside the iterations: median wall time of psk_pcg calls of `short` and of
    max(steps, 200) iterations (no timing events), fitted as T(K) = a + b K; a is what a caller pays
    once per solve (setup launches, final synchronisation, result copies)."""
    N = sys_.N
    steps = max(steps, 10 * short)

    def t(k):
        ts = []
        for _ in range(reps):
            prepared = sys_.args(k, False)
            N.check(N.lib.psk_synchronize(), "sync")
            t0 = time.perf_counter()
            sys_.run(k, False, prepared)
            N.check(N.lib.psk_synchronize(), "sync")
            ts.append(time.perf_counter() - t0)
        return median(ts)
    t_short, t_long = t(short), t(steps)
    b = (t_long - t_short) / (steps - short) if steps > short else float("nan")
    return {"short_iters": short, "long_iters": steps, "short_ms": t_short * 1e3, "long_ms": t_long * 1e3,
            "per_iteration_ms": b * 1e3, "fixed_overhead_ms": (t_short - short * b) * 1e3,
            "short_it_s": short / t_short, "long_it_s": steps / t_long}


def csr_in_loop(sys_, bspmv, steps, repeats=3):
    """The headline solve with the matrix in the CSR layout (PSK_LAYOUT_CSR: the tile kernel with
    LDS-staged products, 80 B/row of SURVEY §8d's CSR bytes): iterations/s and the in-loop CSR SpMV
    priced on the CSR bytes. Leaves the matrix in the CSR layout (call after the other keys)."""
    N = sys_.N
    N.check(N.lib.psk_csr_layout(sys_.A, N.PSK_LAYOUT_CSR, None, None, None, None), "psk_csr_layout")
    sys_.run(5, False)
    regs = []
    for _ in range(repeats):
        prepared = sys_.args(steps, True)
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        res = sys_.run(steps, True, prepared)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append((time.perf_counter() - t0, res.spmv_ms))
    regs.sort()
    dt, sms = regs[len(regs) // 2]
    ach = bspmv / (sms * 1e-3) / 1e9
    return {"kernel": "spmv_kernel<kSpmvDot> (CSR layout, in the PCG loop)", "pcg_it_per_s": steps / dt,
            "spmv_avg_launch_ms": sms, "csr_bytes_per_launch": bspmv, "achieved_GBps": ach,
            "frac": ach / HBM_PEAK_GBPS, "regions_it_s": [steps / r[0] for r in regs]}


class PcgSystem:
    """FDLaplacian2D(-1, 1, m) (row-block shard of this rank when comm is set), its Jacobi
    preconditioner and b = A @ default_rng(12345).random(n), all resident in HBM."""

    def __init__(self, N, m, comm, world):
        self.N = N
        t0 = time.time()
        n, _ = fd_sizes(m)
        self.n = n
        self.A = ctypes.c_void_p()
        if comm is not None:
            rb, re_ = ctypes.c_int64(), ctypes.c_int64()
            N.check(N.lib.psk_csr_create_fd2d_dist(-1.0, 1.0, m, comm, ctypes.byref(self.A), ctypes.byref(rb),
                                                   ctypes.byref(re_)), "psk_csr_create_fd2d_dist")
            row_begin, row_end = rb.value, re_.value
        else:
            N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(self.A)), "psk_csr_create_fd2d")
            row_begin, row_end = 0, n
        self.nloc = row_end - row_begin
        ncols = self.nloc + (m if row_begin > 0 else 0) + (m if row_end < n else 0)
        self.M = ctypes.c_void_p()
        N.check(N.lib.psk_prec_create(self.A, N.PSK_PREC_JACOBI, ctypes.byref(self.M)), "psk_prec_create")
        # x_exact rows of this rank: default_rng(12345).random(n)[row_begin:row_end] (one u64 per double)
        rng = np.random.default_rng(12345)
        rng.bit_generator.advance(row_begin)
        xe = rng.random(self.nloc)
        self.dx, self.db, self.dsol = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        N.check(N.lib.psk_dmalloc(ncols * 8, ctypes.byref(self.dx)), "alloc")
        N.check(N.lib.psk_dmalloc(self.nloc * 8, ctypes.byref(self.db)), "alloc")
        N.check(N.lib.psk_dmalloc(self.nloc * 8, ctypes.byref(self.dsol)), "alloc")
        N.check(N.lib.psk_h2d(self.dx, N.ptr(xe), self.nloc * 8), "h2d")
        del xe
        N.check(N.lib.psk_spmv(self.A, self.dx, self.db, N.PSK_DEVICE), "psk_spmv")   # b = A @ x_exact (halo inside)
        N.check(N.lib.psk_synchronize(), "sync")
        nnz = ctypes.c_int64()
        N.check(N.lib.psk_csr_info(self.A, None, ctypes.byref(nnz)), "info")
        self.nnz_loc = nnz.value
        self.setup_s = time.time() - t0

    def args(self, iters, time_kernels):
        """psk_pcg's control block and result struct (by reference): built before a timed region, so the region
        holds the call itself and not the Python construction of its arguments."""
        N = self.N
        ctl = N.PskCtl(maxiter=iters, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0,
                       time_kernels=EVENT_STRIDE if time_kernels else 0)
        res = N.PskResult()
        return ctl, res, ctypes.byref(ctl), ctypes.byref(res)

    def run(self, iters, time_kernels, prepared=None):
        N = self.N
        _, res, pctl, pres = prepared if prepared is not None else self.args(iters, time_kernels)
        N.check(N.lib.psk_pcg(self.A, self.M, self.db, self.dsol, pctl, pres, None, N.PSK_DEVICE), "psk_pcg")
        return res

    def regions(self, steps, warmup, repeats, barrier, dist, events=True):
        """`repeats` timed regions of exactly `steps` iterations, each bracketed by barrier + device
        sync; per region the max over ranks of (wall time, mean SpMV launch time). events: libpsk
        records HIP events around every SpMV launch (the roofline's kernel time)."""
        N = self.N
        if warmup > 0:   # the same path as the timed regions (the timing events are created here, not in region 1)
            r = self.run(warmup, events)
            assert r.iters == warmup, r.iters
        # then one untimed settle solve of ~0.3 s (a count from n alone, so every rank runs the same), right
        # before the first region: without it the first regions ran slower (round 5: 6033 -> 6282 it/s in order,
        # the SpMV launch 0.061 -> 0.056 ms), and a short solve (W = 5) between it and region 1 still left
        # region 1 ~2% slow (a candidate cause: it writes 6 of the 8 p ring buffers, a 20-iteration one all 8)
        # (profiles/r5_region_order_probe.txt)
        settle = self.settle_iters()
        if settle > 0:
            r = self.run(settle, False)
            assert r.iters == settle, r.iters
        out = []
        self.comm = []   # per region, N > 1: (p.Ap gather ms, halo exchange ms), each the max over ranks
        for _ in range(max(1, repeats)):
            prepared = self.args(steps, events)
            barrier()
            N.check(N.lib.psk_synchronize(), "sync")
            t0 = time.perf_counter()
            res = self.run(steps, events, prepared)
            N.check(N.lib.psk_synchronize(), "sync")
            barrier()
            dt = time.perf_counter() - t0
            LIVE.tick("timed region")
            assert res.iters == steps and res.success == 1, (res.iters, res.success)
            spmv_ms, gat, halo = res.spmv_ms, res.gather_ms, res.halo_ms
            if dist is not None:
                import torch
                t = torch.tensor([dt, spmv_ms, gat, halo], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt, spmv_ms, gat, halo = (float(v) for v in t)
            out.append((dt, spmv_ms, res.spmv_launches))
            self.comm.append((gat, halo, res.comm_samples))
        return out

    def settle_iters(self):
        """Iterations of the settle solve: ~0.3 s at the measured rates (2000 at N = 10M, 74 at 16384^2)."""
        return max(20, min(5000, int(2e10 / max(1, self.n))))

    def layout(self):
        N = self.N
        lay, stream = N.I32(), N.I64()
        N.check(N.lib.psk_csr_layout(self.A, -1, ctypes.byref(lay), None, None, ctypes.byref(stream)),
                "psk_csr_layout")
        return stream.value + 16 * self.nloc, LAYOUT_NAMES[lay.value], lay.value

    def free(self):
        N = self.N
        for p in (self.dx, self.db, self.dsol):
            N.lib.psk_dfree(p)
        N.lib.psk_prec_destroy(self.M)
        N.lib.psk_csr_destroy(self.A)


def median(v):
    s = sorted(v)
    return s[len(s) // 2] if len(s) % 2 else 0.5 * (s[len(s) // 2 - 1] + s[len(s) // 2])


def spmv_kernel_label(layout, mode):
    """Descriptive name of the SpMV kernel a layout runs when no PMC profile of the build names it."""
    if layout == 0:
        return "spmv_kernel<%d> (CSR layout)" % mode
    if LAYOUT_NAMES.get(layout) == "diag":
        return "spmv_diagp_kernel<%d, ...> (diag layout, two rows per lane)" % mode
    return "spmv_uniform(_multi)_kernel / spmv_sliced_kernel <MODE=%d> (%s layout)" % (mode, LAYOUT_NAMES[layout])


def lib_sha256():
    """sha256 of the libpsk.so this process loaded (a PMC profile is only used for the same build)."""
    import hashlib
    from pysolvers_amd import _native as N
    with open(N.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def host_info():
    """nproc, the CPU model name (lscpu's 'Model name' comes from /proc/cpuinfo) and OPENBLAS_NUM_THREADS."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": model,
            "OPENBLAS_NUM_THREADS": os.environ.get("OPENBLAS_NUM_THREADS", "unset (= all cores)"),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS", "unset")}


def cpu_baseline(m, iters):
    """The oracle (op-for-op restatement of PCGSolver.solve, bit-identical to the reference) on the
    host, 1 BLAS thread: a bounded sample of the same workload. iters + 1 iterations run; the first
    (cold) one is dropped and each of the other `iters` is one timed sample; value = 1 / median."""
    from threadpoolctl import threadpool_limits
    from oracle import fdlap, krylov
    t0 = time.time()
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    x = np.random.default_rng(12345).random(m * m)
    b = A @ x
    del x
    setup = time.time() - t0
    marks = []
    with threadpool_limits(limits=1):
        st = krylov.pcg(A, b, maxiter=iters + 1, tau=0.0, fail_on_maxiter=False, precond=krylov.jacobi_form(A),
                        on_iter=lambda k: (marks.append(time.perf_counter()), LIVE.tick("oracle iteration")))
        marks.append(time.perf_counter())
    assert st["iters"] == iters + 1
    per = [marks[k + 1] - marks[k] for k in range(1, iters + 1)]
    return dict(value=1.0 / median(per), unit="CG iterations/s", cores=1, kind="port",
                samples_s_per_iteration=per, host=host_info(),
                sample="%d single-iteration samples (after one untimed iteration) of the oracle's PCG+Jacobi "
                       "(numpy/scipy restatement of PCGSolver.py:64-142, bit-identical to the reference) on the same "
                       "FDLaplacian2D m=%d system, BLAS limited to 1 thread (scipy csr_matvec and numpy ufuncs are "
                       "single-threaded anyway); value = 1 / median sample; %.0f s setup" % (iters, m, setup))


def general_path(N, A, b, x, m, steps, repeats=3):
    """The path a general matrix takes (SpMV layout with double values in slot pairs, DInv streamed
    from HBM) on the same FD system, same iteration count: the headline's value dictionary and
    scalar DInv apply only to constant-coefficient stencils."""
    os.environ["PSK_JACOBI_UNIFORM"] = "0"
    Mg = ctypes.c_void_p()
    try:
        N.check(N.lib.psk_prec_create(A, N.PSK_PREC_JACOBI, ctypes.byref(Mg)), "psk_prec_create")
    finally:
        del os.environ["PSK_JACOBI_UNIFORM"]
    prev = N.I32()
    N.check(N.lib.psk_csr_layout(A, -1, ctypes.byref(prev), None, None, None), "psk_csr_layout")
    N.check(N.lib.psk_csr_layout(A, N.PSK_LAYOUT_SLICED, None, None, None, None), "psk_csr_layout")
    n = m * m

    def run(k, tk):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=tk)
        res = N.PskResult()
        N.check(N.lib.psk_pcg(A, Mg, b, x, ctypes.byref(ctl), ctypes.byref(res), None, N.PSK_DEVICE), "psk_pcg")
        return res
    run(5, 0)
    regs = []
    for _ in range(repeats):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        res = run(steps, 1)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append((time.perf_counter() - t0, res.spmv_ms))
    regs.sort()
    dt, sms = regs[len(regs) // 2]
    bl, lname = layout_bytes(N, A, n)
    vb = vec_bytes_per_row(N, Mg)
    N.lib.psk_prec_destroy(Mg)
    # back to the headline's layout (the later keys time the headline system)
    N.check(N.lib.psk_csr_layout(A, prev.value, None, None, None, None), "psk_csr_layout")
    ach = bl / (sms * 1e-3) / 1e9
    return {"what": "PSK_SPMV_LAYOUT=sliced (double values) + PSK_JACOBI_UNIFORM=0 (streamed DInv), same "
                    "matrix and iteration count; median of %d regions" % repeats,
            "pcg_it_per_s": steps / dt, "ms_per_step": dt * 1e3 / steps, "layout": lname,
            "spmv_avg_launch_ms": sms, "spmv_algorithmic_bytes_per_launch": bl, "spmv_achieved_GBps": ach,
            "spmv_frac": ach / HBM_PEAK_GBPS, "vector_bytes_per_row": vb,
            "pcg_iteration_frac_of_peak": (bl + vb * n) * steps / dt / 1e9 / HBM_PEAK_GBPS}


def csr_layout_batch(N, A, x, y, bspmv, reps=20):
    """The same matrix switched to the CSR layout (tile kernel, LDS-staged products) and multiplied
    `reps` times back to back: the CSR SpMV the north star names, beside the default layout. The
    matrix is left in CSR layout afterwards (call last)."""
    N.check(N.lib.psk_csr_layout(A, N.PSK_LAYOUT_CSR, None, None, None, None), "psk_csr_layout")
    ms = ctypes.c_double()
    N.check(N.lib.psk_spmv_timed(A, x, y, reps, ctypes.byref(ms)), "psk_spmv_timed")
    gbps = bspmv / (ms.value * 1e-3) / 1e9
    return {"kernel": "spmv_kernel<kSpmvPlain> (CSR layout)", "avg_launch_ms": ms.value, "achieved_GBps": gbps,
            "frac": gbps / HBM_PEAK_GBPS}


def pmc_traffic(path, m, world, mode, sliced):
    """HBM bytes per launch of the SpMV kernel of mode `mode` (1 = kSpmvDot, the PCG loop's; 0 =
    plain) measured by rocprofv3 PMC passes of THIS build at the same side (scripts/gpu_pmc.sh ->
    tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE, gfx950 corrections calibrated by
    tools/pmc_calib.hip). The profile must record the sha256 of the same libpsk.so and hold exactly
    one SpMV kernel of that mode; otherwise traffic is null and the reason is given. Counters
    cannot be read from inside the timed run."""
    import re
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {"traffic": None, "traffic_note": "no PMC profile at %s" % os.path.relpath(path, REPO)}
    src = os.path.relpath(path, REPO)
    if d.get("config", {}).get("side") != m or world != 1:
        return {"traffic": None, "traffic_note": "%s is for another side / rank count" % src}
    if d.get("libpsk_sha256") != lib_sha256():
        return {"traffic": None, "traffic_note": "%s was captured with another libpsk.so build" % src}
    pat = re.compile((r"psk::spmv_(uniform_multi|uniform|sliced|diag|diagp)_kernel<%d," if sliced else r"psk::spmv_kernel<%d>") % mode)
    hits = [k for k in d["kernels"] if pat.search(k)]
    if len(hits) != 1:
        return {"traffic": None, "traffic_note": "%s holds %d SpMV kernels of mode %d" % (src, len(hits), mode)}
    v = d["kernels"][hits[0]]
    return {"kernel": hits[0].split("(")[0].replace("void ", ""), "traffic": v["hbm_bytes_per_launch"],
            "traffic_source": "%s (rocprofv3 PMC FETCH_SIZE/WRITE_SIZE passes, same libpsk.so sha256, "
                              "%d launches)" % (src, v["launches"])}


def pcg_4096(N, iters=300):
    """configs[1]: PCG+Jacobi on FDLaplacian2D 4096^2, one GPU, `iters` fixed iterations (median of 5)."""
    m = 4096
    n, nnz = fd_sizes(m)
    A, M, db, dx = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "fd2d")
    N.check(N.lib.psk_prec_create(A, N.PSK_PREC_JACOBI, ctypes.byref(M)), "prec")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(db)), "alloc")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dx)), "alloc")
    xe = np.random.default_rng(12345).random(n)
    N.check(N.lib.psk_h2d(dx, N.ptr(xe), n * 8), "h2d")
    N.check(N.lib.psk_spmv(A, dx, db, N.PSK_DEVICE), "spmv")

    def run(k, tk):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=tk)
        res = N.PskResult()
        N.check(N.lib.psk_pcg(A, M, db, dx, ctypes.byref(ctl), ctypes.byref(res), None, N.PSK_DEVICE), "pcg")
        return res
    run(20, 0)
    regs = []
    for _ in range(5):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        run(iters, 0)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append(time.perf_counter() - t0)
    dt = median(regs)
    res = run(50, 1)
    bl, lname = layout_bytes(N, A, n)
    out = {"n": n, "nnz": nnz, "iters": iters, "layout": lname, "pcg_it_per_s": iters / dt,
           "regions_it_s": [iters / r for r in regs],
           "pcg_iteration_frac_of_peak": (bl + vec_bytes_per_row(N, M) * n) * iters / dt / 1e9 / HBM_PEAK_GBPS,
           "spmv_avg_launch_ms": res.spmv_ms, "spmv_frac": bl / (res.spmv_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    for p in (db, dx):
        N.lib.psk_dfree(p)
    N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(A)
    return out


def gmres_arnoldi(N, m=4096, restart=30, cycles=2, repeats=3):
    """GMRES(30) + Jacobi on FDLaplacian2D 4096^2, one GPU: Arnoldi steps/s over exactly `cycles`
    restart cycles per timed solve (tau = 0), priced on two byte models per step k (k = 0..29):
      * reference op list: B_spmv(CSR) + (k+1) 40n + 24n, + 24n for the Jacobi apply;
      * libpsk's fused schedule: the SpMV layout's stream + x and DInv gathers + y written + q_0 read
        (layout bytes + 16n; Jacobi fused into the gather), MGS j < k 32n (u read + written, q_j and
        q_{j+1} read), j = k 24n, normalisation 16n (u read, q_{k+1} written): layout + (56 + 32k) n.
    The restart (host least-squares solve, x update, residual SpMV) is inside the timed region."""
    n, nnz = fd_sizes(m)
    A, M, db, dx = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "fd2d")
    os.environ["PSK_JACOBI_UNIFORM"] = "0"
    try:
        N.check(N.lib.psk_prec_create(A, N.PSK_PREC_JACOBI, ctypes.byref(M)), "prec")
    finally:
        del os.environ["PSK_JACOBI_UNIFORM"]
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(db)), "alloc")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dx)), "alloc")
    xe = np.random.default_rng(12345).random(n)
    N.check(N.lib.psk_h2d(dx, N.ptr(xe), n * 8), "h2d")
    N.check(N.lib.psk_spmv(A, dx, db, N.PSK_DEVICE), "spmv")
    steps = restart * cycles

    def run(k):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=restart, check_every=0, time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_gmres(A, M, db, dx, ctypes.byref(ctl), ctypes.byref(res), None, N.PSK_DEVICE), "psk_gmres")
        return res
    run(restart)
    regs = []
    for _ in range(repeats):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        run(steps)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append(time.perf_counter() - t0)
    dt = median(regs)
    bl, lname = layout_bytes(N, A, n)
    ks = range(restart)
    b_ref = sum(spmv_bytes(n, nnz) + (k + 1) * 40 * n + 24 * n + 24 * n for k in ks) / restart
    b_fused = sum(bl + 16 * n + (56 + 32 * k) * n for k in ks) / restart
    sps = steps / dt
    out = {"workload": "GMRES(%d) + Jacobi, FDLaplacian2D %dx%d, tau=0, %d Arnoldi steps (%d cycles) per solve, "
                       "median of %d" % (restart, m, m, steps, cycles, repeats),
           "n": n, "layout": lname, "steps_per_s": sps, "ms_per_step": dt * 1e3 / steps,
           "regions_steps_per_s": [steps / r for r in regs],
           "bytes_per_step_reference_ops": b_ref, "bytes_per_step_fused": b_fused,
           # the reference's op list moves more bytes than the fused kernels do, so its count over the
           # measured time is NOT a bandwidth (it can exceed the peak); frac_fused is the roofline figure
           "reference_ops_count_over_time_GBps": b_ref * sps / 1e9,
           "frac_fused": b_fused * sps / 1e9 / HBM_PEAK_GBPS}
    for p in (db, dx):
        N.lib.psk_dfree(p)
    N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(A)
    return out


def trisolve_schedules(N, h):
    """Schedule the library chose for each factor of a triangular-solve chain."""
    names = {0: "syncfree", 1: "band", 2: "lds", 3: "grid", 4: "part", 5: "strip"}
    out = []
    for which in (0, 1):
        s, blocks = N.I32(), N.I64()
        N.check(N.lib.psk_prec_trisolve_schedule(h, which, -1, ctypes.byref(s), ctypes.byref(blocks), None, None,
                                                 None), "psk_prec_trisolve_schedule")
        out.append(names.get(s.value, s.value))
    return out


def gmres_ilut(N, m=2896, restart=30, steps=60, repeats=3):
    """configs[2]: GMRES(30) + right ILUT (the reference's spilu arguments, ILUTPreconditioner.py:51-53)
    on FDLaplacian2D m^2, one GPU, exactly `steps` Arnoldi steps per timed solve (tau = 0). m = 2896
    is the largest side scipy's SuperLU forms this ILUT for (4096^2: SUPERLU_MALLOC fails, in the
    reference too; profiles/r1_gmres_ilut_4096_unformable.json). Latency model: the ILU apply is two
    dependency chains; us_per_level = apply time / (levels of L + levels of U)."""
    import pysolvers_amd as psk
    n = m * m
    t = time.time()
    dA = psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m)
    x = psk.DeviceVector.from_numpy(np.random.default_rng(12345).random(n))
    b = psk.Linear.spmv(dA, x)
    del x
    out = {"workload": "GMRES(%d) + RightILUT(drop_tol=1e-3, fill_factor=15), FDLaplacian2D %dx%d, tau=0, %d Arnoldi "
                       "steps per solve" % (restart, m, m, steps), "n": n}
    try:
        M = psk.RightILUT().form(dA)
    except RuntimeError as e:
        out["error"] = "reference ILUT factorization failed: %s" % e
        return out
    out["ilut_setup_s"] = time.time() - t
    progress("configs2_gmres30_ilut: device solves")
    info = M.device_info()
    out.update(nnz_L=info["nnz_l"], nnz_U=info["nnz_u"], levels_L=info["levels_l"], levels_U=info["levels_u"],
               schedules=trisolve_schedules(N, M.device_handle))
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
    M.applyRight(v)
    ap = []
    for _ in range(5):
        N.check(N.lib.psk_synchronize(), "sync")
        t2 = time.perf_counter()
        M.applyRight(v)
        N.check(N.lib.psk_synchronize(), "sync")
        ap.append((time.perf_counter() - t2) * 1e3)
    apply_ms = median(ap)
    ilu_bytes = 12 * (info["nnz_l"] + info["nnz_u"]) + 80 * n
    out["ilu_apply"] = {"bound": "latency (dependency chain)", "ms": apply_ms,
                        "us_per_level": apply_ms * 1e3 / max(1, info["levels_l"] + info["levels_u"]),
                        "bytes_model": "12 B per factor entry + 80 B per row (gathers, rhs, diagonal, x)",
                        "bytes": ilu_bytes, "achieved_GBps": ilu_bytes / (apply_ms * 1e-3) / 1e9,
                        "frac_of_hbm_peak": ilu_bytes / (apply_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    sol = psk.DeviceVector(n)

    def run(k):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=restart, check_every=0, time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_gmres(dA.handle, M.device_handle, b._p, sol._p, ctypes.byref(ctl), ctypes.byref(res), None,
                                N.PSK_DEVICE), "psk_gmres")
        return res
    run(restart)
    regs = []
    for _ in range(repeats):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        res = run(steps)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append(time.perf_counter() - t0)
    dt = median(regs)
    out.update(steps_per_s=steps / dt, ms_per_step=dt * 1e3 / steps, regions_steps_per_s=[steps / r for r in regs],
               ilu_share_of_step=apply_ms / (dt * 1e3 / steps), status=int(res.status),
               rec_resid_ratio=res.resid_recursive / res.norm_b, setup_s=time.time() - t)
    return out


def pcg_amg(N, m=8192, levels=5, cycles=2, iters=6, repeats=3):
    """configs[4]: PCG + AMG(numIters=2, 5 levels, Gauss-Seidel nu = 2 + 2) on -FDLaplacian2D m^2 (the
    sign FDBratu2D.py:15 uses), one GPU, exactly `iters` PCG iterations per timed solve (PCG+AMG does
    not converge on this matrix). Latency model: each apply runs cycles x (nuPre +
    nuPost) fine Gauss-Seidel sweeps, each a dependency chain of 2m - 1 levels."""
    import pysolvers_amd as psk
    n = m * m
    t = time.time()
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    dA = psk.DeviceCSR.from_scipy(A)
    x = psk.DeviceVector.from_numpy(np.random.default_rng(12345).random(n))
    b = psk.Linear.spmv(dA, x)
    del x
    out = {"workload": "PCG + AMG(numIters=%d, numLevels=%d, nuPre=2, nuPost=2, GaussSeidelSmoother), "
                       "-FDLaplacian2D %dx%d, tau=0, %d iterations per solve" % (cycles, levels, m, m, iters), "n": n}
    t1 = time.time()
    M = psk.AMG(numIters=cycles, numLevels=levels, smoother=psk.GaussSeidelSmoother).form(dA)
    del A
    out["amg_setup_s"] = time.time() - t1
    progress("configs4_pcg_amg_8192: device solves")
    out["level_sizes"] = M.levels()
    out["coarse_solve"] = M.coarse_kind   # dense: streamed GEMV over A_c^-1 (dense.hip); lu: SuperLU factors

    def timed(fn, reps=3):
        fn()
        ts = []
        for _ in range(reps):
            N.check(N.lib.psk_synchronize(), "sync")
            t2 = time.perf_counter()
            fn()
            N.check(N.lib.psk_synchronize(), "sync")
            ts.append((time.perf_counter() - t2) * 1e3)
        return median(ts)
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(n))
    out["amg_apply_ms"] = timed(lambda: M.apply(v))
    S = M._S[-1].operator
    fine_levels = S.device_info()["levels_u"]
    sweep_ms = timed(lambda: S.apply(v))
    # one serialized sweep (the smoother's own apply); inside the V-cycle the fine level's sweeps run two per launch
    # (amg.hip gs_pair_kernel: nuPre = nuPost = 2 -> one launch each), bit-identical to these
    out["fine_gs_sweep"] = {"bound": "latency (dependency chain)", "ms": sweep_ms, "dep_levels": fine_levels,
                            "us_per_level": sweep_ms * 1e3 / max(1, fine_levels),
                            "schedule": S.schedule("U")["schedule"],
                            "sweeps_per_apply": cycles * 4,
                            "in_apply": "two sweeps per launch (gs_pair_kernel), %d launches" % (cycles * 2)}
    co = M._coarse
    v0 = psk.DeviceVector.from_numpy(np.random.default_rng(0).standard_normal(M.levels()[0]))
    out["coarse_solve_ms"] = timed(lambda: co.apply(v0))
    sol = psk.DeviceVector(n)

    def run(k):
        ctl = N.PskCtl(maxiter=k, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=0)
        res = N.PskResult()
        N.check(N.lib.psk_pcg(dA.handle, M.device_handle, b._p, sol._p, ctypes.byref(ctl), ctypes.byref(res), None,
                              N.PSK_DEVICE), "psk_pcg")
        return res
    run(1)
    regs = []
    for _ in range(repeats):
        N.check(N.lib.psk_synchronize(), "sync")
        t0 = time.perf_counter()
        res = run(iters)
        N.check(N.lib.psk_synchronize(), "sync")
        regs.append(time.perf_counter() - t0)
    dt = median(regs)
    out.update(pcg_it_per_s=iters / dt, ms_per_it=dt * 1e3 / iters, regions_it_s=[iters / r for r in regs],
               status=int(res.status), iters_done=int(res.iters), setup_s=time.time() - t)
    return out


if __name__ == "__main__":
    main()
