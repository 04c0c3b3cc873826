#!/usr/bin/env python3
"""Benchmark: PCG + Jacobi iterations/s on the 5-point FDLaplacian2D, CSR SpMV vs the HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--side M]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one PCG iteration (PCGSolver.py:109-138: SpMV, 2 dots + norm, 3 updates, Jacobi
apply) over the whole matrix. The workload is fixed for every N (strong scaling): A =
FDLaplacian2D(-1, 1, m) generated on the device (bit-identical to examples/FDLaplacian2D.py),
b = A @ default_rng(12345).random(n), control = CommonSolverArgs(maxiter=K, tau=0,
failOnMaxiter=False) so exactly K iterations run (PCGSolver.py:129-131). With N > 1 the rows are
split on whole grid lines across ranks (one process per GPU), halo lines are exchanged with
ncclSend/Recv and the dot partials all-reduced with RCCL over xGMI, all inside libpsk.

Timed region: barrier + device sync, ONE psk_pcg call of K iterations, device sync + barrier;
max over ranks. `roofline` prices the SpMV kernel (the dominant kernel) from HIP events
recorded by libpsk on its own stream around every SpMV launch of the timed solve.
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
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def fd_sizes(m):
    n = m * m
    nnz = 1 if m == 1 else 5 * n - 4 * m
    return n, nnz


def spmv_bytes(n, nnz):
    """Algorithmic SpMV bytes: vals+colidx, rowptr, x once, y written."""
    return 12 * nnz + 4 * (n + 1) + 16 * n


PCG_VEC_BYTES_PER_ROW = 80   # K2 (r, Ap, dinv in; r out) + K3 (r, p, x, dinv in; x, p out), Jacobi
LAYOUT_NAMES = {0: "csr", 1: "sliced", 2: "sliced_wide", 3: "sliced_dict"}   # PSK_LAYOUT_*


def pcg_iter_bytes(n, nnz, jacobi=True):
    """Compulsory bytes of one PCG iteration in libpsk's 3-launch schedule with a CSR SpMV
    (SURVEY.md §8d)."""
    return spmv_bytes(n, nnz) + (PCG_VEC_BYTES_PER_ROW if jacobi else 64) * n


def vec_bytes_per_row(N, M):
    """K2 + K3 bytes per row: 80 with a streamed DInv, 64 when the Jacobi diagonal is one scalar
    (psk_prec_jacobi_uniform)."""
    u = N.I32()
    N.check(N.lib.psk_prec_jacobi_uniform(M, ctypes.byref(u), None), "psk_prec_jacobi_uniform")
    return PCG_VEC_BYTES_PER_ROW - (16 if u.value else 0)


def layout_bytes(N, A, n):
    """Bytes one SpMV of A must move in its current storage layout — the matrix stream
    (psk_csr_layout) + x read once + y written — and the layout's name."""
    lay, stream = N.I32(), N.I64()
    N.check(N.lib.psk_csr_layout(A, -1, ctypes.byref(lay), None, None, ctypes.byref(stream)), "psk_csr_layout")
    return stream.value + 16 * n, LAYOUT_NAMES[lay.value]


def cpu_baseline(m, iters):
    """The oracle (op-for-op restatement of PCGSolver.solve, bit-identical to the reference) on the
    host, 1 BLAS thread: a bounded sample of `iters` iterations of the same workload."""
    from threadpoolctl import threadpool_limits
    from oracle import fdlap, krylov
    t0 = time.time()
    A = fdlap.fd_laplacian_2d(-1.0, 1.0, m)
    x = np.random.default_rng(12345).random(m * m)
    b = A @ x
    del x
    setup = time.time() - t0
    with threadpool_limits(limits=1):
        t = time.perf_counter()
        st = krylov.pcg(A, b, maxiter=iters, tau=0.0, fail_on_maxiter=False, precond=krylov.jacobi_form(A))
        dt = time.perf_counter() - t
    assert st["iters"] == iters
    return dict(value=iters / dt, unit="CG iterations/s", cores=1, kind="port",
                sample="%d PCG+Jacobi iterations of the oracle (numpy/scipy restatement of PCGSolver.py:64-142, "
                       "bit-identical to the reference) on the same FDLaplacian2D m=%d system, 1 BLAS thread; "
                       "%.1f s timed, %.0f s setup" % (iters, m, dt, setup))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--side", type=int, default=16384, help="grid side m of FDLaplacian2D (n = m^2 rows)")
    ap.add_argument("--cpu-iters", type=int, default=2, help="oracle iterations for cpu_baseline (0 = skip)")
    ap.add_argument("--spmv10m", type=int, default=1, help="also time SpMV at N=10M (m=3163) on rank 0")
    ap.add_argument("--config1", type=int, default=1, help="also time configs[1] (PCG+Jacobi 4096^2) on rank 0")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r1h_pmc_traffic_16384.json"),
                    help="PMC traffic summary (tools/pmc_summary.py) of the same kernel and side")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))

    from pysolvers_amd import _native as N
    # one GPU per rank: LOCAL_RANK when every GPU is visible to every rank; a launcher that narrows
    # visibility per rank leaves one device (ordinal 0) per process
    ndev = N.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    dev = int(os.environ.get("PSK_BENCH_DEVICE", local_rank if local_rank < ndev else local_rank % ndev))
    N.check(N.lib.psk_set_device(dev), "psk_set_device")

    dist = None
    if world > 1:
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

    m = args.side
    n, nnz = fd_sizes(m)
    t_setup = time.time()
    # ---- operator, preconditioner, right-hand side (all resident in HBM before timing) -----------
    comm = ctypes.c_void_p()
    A = ctypes.c_void_p()
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
    if world > 1:
        rb, re_ = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib.psk_csr_create_fd2d_dist(-1.0, 1.0, m, comm, ctypes.byref(A), ctypes.byref(rb),
                                               ctypes.byref(re_)), "psk_csr_create_fd2d_dist")
        row_begin, row_end = rb.value, re_.value
    else:
        N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "psk_csr_create_fd2d")
        row_begin, row_end = 0, n
    nloc = row_end - row_begin
    ncols = nloc + (m if row_begin > 0 else 0) + (m if row_end < n else 0)
    M = ctypes.c_void_p()
    N.check(N.lib.psk_prec_create(A, N.PSK_PREC_JACOBI, ctypes.byref(M)), "psk_prec_create")
    # x_exact rows of this rank: default_rng(12345).random(n)[row_begin:row_end] (one u64 per double)
    rng = np.random.default_rng(12345)
    rng.bit_generator.advance(row_begin)
    xe = rng.random(nloc)
    dx = ctypes.c_void_p()
    db = ctypes.c_void_p()
    dsol = ctypes.c_void_p()
    N.check(N.lib.psk_dmalloc(ncols * 8, ctypes.byref(dx)), "alloc")
    N.check(N.lib.psk_dmalloc(nloc * 8, ctypes.byref(db)), "alloc")
    N.check(N.lib.psk_dmalloc(nloc * 8, ctypes.byref(dsol)), "alloc")
    N.check(N.lib.psk_h2d(dx, N.ptr(xe), nloc * 8), "h2d")
    del xe
    N.check(N.lib.psk_spmv(A, dx, db, N.PSK_DEVICE), "psk_spmv")      # b = A @ x_exact (halo inside)
    N.check(N.lib.psk_synchronize(), "sync")
    setup_s = time.time() - t_setup

    def run(iters, time_kernels):
        ctl = N.PskCtl(maxiter=iters, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0,
                       time_kernels=int(time_kernels))
        res = N.PskResult()
        N.check(N.lib.psk_pcg(A, M, db, dsol, ctypes.byref(ctl), ctypes.byref(res), None, N.PSK_DEVICE), "psk_pcg")
        return res

    if args.warmup > 0:
        r = run(args.warmup, False)
        assert r.iters == args.warmup, r.iters
    barrier()
    N.check(N.lib.psk_synchronize(), "sync")
    t0 = time.perf_counter()
    res = run(args.steps, True)
    N.check(N.lib.psk_synchronize(), "sync")
    barrier()
    dt = time.perf_counter() - t0
    assert res.iters == args.steps and res.success == 1, (res.iters, res.success)
    if dist is not None:
        import torch
        t = torch.tensor([dt, res.spmv_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, spmv_ms_max = float(t[0]), float(t[1])
    else:
        spmv_ms_max = res.spmv_ms

    if rank == 0:
        it_s = args.steps / dt
        nloc_r0 = nloc
        nnz_loc = ctypes.c_int64()
        N.check(N.lib.psk_csr_info(A, None, ctypes.byref(nnz_loc)), "info")
        bspmv = spmv_bytes(nloc_r0, nnz_loc.value)
        lay, slots, packed, stream = N.I32(), N.I64(), N.I64(), N.I64()
        N.check(N.lib.psk_csr_layout(A, -1, ctypes.byref(lay), ctypes.byref(slots), ctypes.byref(packed),
                                     ctypes.byref(stream)), "psk_csr_layout")
        sliced = lay.value != N.PSK_LAYOUT_CSR
        kname = "spmv_sliced_kernel<kSpmvDot>" if sliced else "spmv_kernel<kSpmvDot>"
        # the bytes this launch must move in its storage layout (matrix stream + x read + y written;
        # DESIGN.md "Roofline accounting"); with a value dictionary far fewer than CSR's 12 B/entry
        blay = stream.value + 16 * nloc_r0
        ach = blay / (res.spmv_ms * 1e-3) / 1e9 if res.spmv_ms > 0 else None
        csr_eq = bspmv / (res.spmv_ms * 1e-3) / 1e9 if res.spmv_ms > 0 else None
        vb = vec_bytes_per_row(N, M)
        biter = blay * world + vb * n
        out = {
            "metric": METRIC,
            "value": it_s,
            "unit": "CG iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: FDLaplacian2D(-1,1,m) built on device (bit-identical to the reference "
                    "generator), b = A @ default_rng(12345).random(n)",
            "config": {"workload": "PCG+Jacobi, FDLaplacian2D %dx%d (n=%d, nnz=%d), tau=0 fixed-iteration"
                                   % (m, m, n, nnz),
                       "m": m, "precond": "jacobi", "parallelism": "row-block x%d (%s)" % (world, "RCCL" if transport == "rccl" else "host-shm rehearsal")
                       if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "kernel": kname + " (rank 0)",
                         "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": (ach / HBM_PEAK_GBPS) if ach else None,
                         **pmc_traffic(args.traffic_json, m, world, sliced),
                         "algorithmic_bytes_per_launch": blay, "avg_launch_ms": res.spmv_ms,
                         "launches": res.spmv_launches, "layout": LAYOUT_NAMES[lay.value],
                         "csr_bytes_per_launch": bspmv, "csr_equivalent_GBps": csr_eq},
            "pcg_iteration_roofline": {"bytes_per_iteration": biter, "vector_bytes_per_row": vb,
                                       "achieved_GBps": biter * it_s / 1e9,
                                       "frac_of_aggregate_peak": biter * it_s / 1e9 / (HBM_PEAK_GBPS * world)},
            "setup_s": setup_s,
        }
        if world == 1:
            # the same matrix, plain y = A x launches back to back (no dot epilogue, no solver kernels
            # in between): how much of the in-loop SpMV time is the PCG context
            bms = ctypes.c_double()
            N.check(N.lib.psk_spmv_timed(A, db, dsol, 20, ctypes.byref(bms)), "psk_spmv_timed")
            out["spmv_plain_batch20"] = {"avg_launch_ms": bms.value,
                                         "achieved_GBps": blay / (bms.value * 1e-3) / 1e9,
                                         "frac": blay / (bms.value * 1e-3) / 1e9 / HBM_PEAK_GBPS}
            out["spmv_csr_layout_batch20"] = csr_layout_batch(N, A, db, dsol, bspmv)
        if transport == "host" and world > 1:
            out["rehearsal"] = "PSK_BENCH_TRANSPORT=host: all ranks on one GPU, host shared-memory collectives; not a measurement"
        if world == 1 and args.spmv10m and m != 3163:
            out["spmv_N10M"] = spmv_10m(N)
        if world == 1 and args.config1 and m != 4096:
            out["configs1_pcg_jacobi_4096"] = pcg_4096(N)
        if world == 1 and args.cpu_iters > 0:
            cb = cpu_baseline(m, args.cpu_iters)
            cb["threads_note"] = "scipy csr_matvec and numpy ufuncs are single-threaded; BLAS limited to 1"
            out["cpu_baseline"] = cb
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)

    N.lib.psk_dfree(dx)
    N.lib.psk_dfree(db)
    N.lib.psk_dfree(dsol)
    N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(A)
    if world > 1:
        barrier()
        N.lib.psk_comm_destroy(comm)
        dist.destroy_process_group()


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


def pmc_traffic(path, m, world, sliced):
    """HBM bytes per SpMV launch measured by rocprofv3 PMC passes on the same kernel and matrix
    (scripts/gpu_pmc.sh -> tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE, gfx950 corrections
    calibrated by tools/pmc_calib.hip). Counters cannot be read from inside the timed run."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {"traffic": None}
    if d.get("config", {}).get("side") != m or world != 1:
        return {"traffic": None}
    # kSpmvDot = 1; the sliced kernel's second template argument is the dictionary size class
    want = ("void psk::spmv_sliced_kernel<1>", "void psk::spmv_sliced_kernel<1,") if sliced \
        else ("void psk::spmv_kernel<1>",)
    for k, v in d["kernels"].items():
        if k.startswith(want):
            return {"traffic": v["hbm_bytes_per_launch"],
                    "traffic_source": os.path.relpath(path, REPO) + " (rocprofv3 PMC, same kernel/config)"}
    return {"traffic": None}


def spmv_10m(N, iters=30):
    """SpMV at the metric's N=10M (m=3163): mean launch time of the PCG SpMV over `iters` iterations."""
    m = 3163
    n, nnz = fd_sizes(m)
    A, M, db, dx = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "fd2d")
    N.check(N.lib.psk_prec_create(A, N.PSK_PREC_JACOBI, ctypes.byref(M)), "prec")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(db)), "alloc")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dx)), "alloc")
    xe = np.random.default_rng(12345).random(n)
    N.check(N.lib.psk_h2d(dx, N.ptr(xe), n * 8), "h2d")
    N.check(N.lib.psk_spmv(A, dx, db, N.PSK_DEVICE), "spmv")
    ctl = N.PskCtl(maxiter=iters, tau=0.0, fail_on_maxiter=0, restart=0, check_every=0, time_kernels=1)
    res = N.PskResult()
    N.check(N.lib.psk_pcg(A, M, db, dx, ctypes.byref(ctl), ctypes.byref(res), None, N.PSK_DEVICE), "pcg")
    b = spmv_bytes(n, nnz)
    bl, lname = layout_bytes(N, A, n)
    gbps = bl / (res.spmv_ms * 1e-3) / 1e9
    # back-to-back launches between two events (no per-launch event in between)
    bms = ctypes.c_double()
    N.check(N.lib.psk_spmv_timed(A, dx, db, 50, ctypes.byref(bms)), "psk_spmv_timed")
    bb = bl / (bms.value * 1e-3) / 1e9
    csr = csr_layout_batch(N, A, dx, db, b, reps=50)
    out = {"n": n, "nnz": nnz, "layout": lname, "avg_launch_ms": res.spmv_ms, "achieved_GBps": gbps,
           "frac": gbps / HBM_PEAK_GBPS, "pcg_it_per_s": iters / (res.loop_ms * 1e-3),
           "algorithmic_bytes_per_launch": bl, "csr_bytes_per_launch": b,
           "csr_equivalent_GBps": b / (res.spmv_ms * 1e-3) / 1e9,
           "batch50": {"kernel": "SpMV, plain mode, the matrix's default layout", "avg_launch_ms": bms.value, "achieved_GBps": bb,
                       "frac": bb / HBM_PEAK_GBPS,
                       "how": "50 back-to-back launches between two HIP events on the library stream"},
           "batch50_csr_layout": csr}
    for p in (db, dx):
        N.lib.psk_dfree(p)
    N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(A)
    return out


def pcg_4096(N, iters=300):
    """configs[1]: PCG+Jacobi on FDLaplacian2D 4096^2, one GPU, `iters` fixed iterations."""
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
    N.check(N.lib.psk_synchronize(), "sync")
    t0 = time.perf_counter()
    run(iters, 0)
    N.check(N.lib.psk_synchronize(), "sync")
    dt = time.perf_counter() - t0
    res = run(50, 1)
    bl, lname = layout_bytes(N, A, n)
    out = {"n": n, "nnz": nnz, "iters": iters, "layout": lname, "pcg_it_per_s": iters / dt,
           "pcg_iteration_frac_of_peak": (bl + vec_bytes_per_row(N, M) * n) * iters / dt / 1e9 / HBM_PEAK_GBPS,
           "spmv_avg_launch_ms": res.spmv_ms, "spmv_frac": bl / (res.spmv_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    for p in (db, dx):
        N.lib.psk_dfree(p)
    N.lib.psk_prec_destroy(M)
    N.lib.psk_csr_destroy(A)
    return out


if __name__ == "__main__":
    main()
