// dense.hip — the AMG coarse-level direct solve as a streamed dense inverse (round 5).
//
// The reference solves the coarsest level with spsolve(A_c, f) on every V-cycle (VCycleManager.py:34-37).
// Through round 4 that was the SuperLU factors of A_c run as two sparse triangular solves: at -FD 8192^2
// (5 levels, A_c 16,642 x 16,642) one workgroup walks 6,016 dependency levels, 4.84 ms per solve. Here
// A_c^-1 is formed once on the device (rocSOLVER getrf + getri, loaded on first use) and each solve is
// one GEMV over it: 16,642^2 x 8 B = 2.2 GB streamed from HBM at close to its bandwidth (~0.4 ms), with
// no dependency chain at all. Optionally one refinement step x += A_c^-1 (f - A_c x) (a sparse SpMV and
// a second GEMV); the single GEMV already agrees with the SuperLU solve to ~2e-15 relative on the SA
// coarse operators of the Laplacian (tests/test_gpu_amg.py pins 1e-12), so refinement is off by default.
//
// Layout: M row-major with row pitch ld (a multiple of 8 doubles, rows 64-B aligned). rocSOLVER works on
// column-major matrices: the row-major image of A_c is the column-major image of A_c^T, whose inverse
// (A_c^T)^-1 read back row-major is A_c^-1 — no transpose pass.
//
// GEMV (dense_gemv_kernel): work units of kDenseRows rows x kDenseCols columns (one workgroup each, two
// rows per wave, so every f load feeds two rows). A unit's row partials go to part[seg][row]; the
// workgroup drawing a row block's last ticket sums its nseg partials in segment order, so y is
// bitwise reproducible whatever order the units run in. Units of 128 KiB give ~18,700 workgroups at
// n = 16,642: the dispatcher deals them as CUs free up, so no CU is left with a long tail.
#include "psk_internal.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>

namespace psk {

constexpr int kDenseRowsPerWave = 2;
constexpr int kDenseRows = kDenseRowsPerWave * kWaves;   // rows of a unit (8)
constexpr int kDenseCols = 2048;                          // columns of a unit (16 KiB of a row)
constexpr int kDenseBatch = 4;                            // double2 loads per row in flight per lane
constexpr int kDenseCntStride = 16;                       // row-block counters 64 B apart

struct DenseInverse {
    double *M = nullptr;   // n x ld, row-major, A^-1
    int64_t ld = 0;
    int32_t nseg = 0;      // column segments
    int64_t nrb = 0;       // row blocks
    uint64_t *part = nullptr;   // nseg * n partials (nseg > 1)
    uint32_t *cnt = nullptr;    // nrb counters (zero between launches)
    int32_t *err = nullptr;     // set when a partial never landed (bounded wait; dense_check_error)
    double *work = nullptr;     // 2 ld: x1, r (refinement)
    const psk_csr *A = nullptr; // borrowed: the refinement's residual
    int32_t refine = 0;
};

void dense_free(DenseInverse *d) {
    if (!d) return;
    void *ptrs[] = {d->M, d->part, d->cnt, d->work, d->err};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete d;
}

// D[i*ld + col] += a_ik for the row's entries in stored order (duplicates summed)
__global__ void dense_scatter_kernel(int64_t n, int64_t ld, const int32_t *__restrict__ rowptr,
                                     const int32_t *__restrict__ colidx, const double *__restrict__ vals,
                                     double *__restrict__ D) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double *row = D + i * ld;
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) row[colidx[k]] += vals[k];
}

// y = M f (+ add): see the header. Grid = nrb * nseg units, unit b = (row block b / nseg, segment b % nseg).
template <bool ADD>
__global__ __launch_bounds__(kBlock) void dense_gemv_kernel(int64_t n, int64_t ld, int32_t nseg,
                                                            const double *__restrict__ M,
                                                            const double *__restrict__ f,
                                                            const double *add, double *y,
                                                            uint64_t *__restrict__ part, uint32_t *__restrict__ cnt,
                                                            int32_t *err) {
    const int64_t b = blockIdx.x, rb = b / nseg;
    const int32_t seg = (int32_t)(b - rb * nseg);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r0 = rb * kDenseRows + wave * kDenseRowsPerWave, r1 = r0 + 1;
    const double *m0 = M + std::min(r0, n - 1) * ld, *m1 = M + std::min(r1, n - 1) * ld;
    const int64_t c0 = (int64_t)seg * kDenseCols, cend = std::min<int64_t>(c0 + kDenseCols, n);
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;   // row r0 even/odd columns, row r1 even/odd columns
    if (cend - c0 == kDenseCols) {
#pragma unroll
        for (int k0 = 0; k0 < kDenseCols / 128; k0 += kDenseBatch) {
            dv2 fv[kDenseBatch], x0[kDenseBatch], x1[kDenseBatch];
#pragma unroll
            for (int j = 0; j < kDenseBatch; ++j) {
                const int64_t c = c0 + (k0 + j) * 128 + lane * 2;
                x0[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(m0 + c));
                x1[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(m1 + c));
                fv[j] = *reinterpret_cast<const dv2 *>(f + c);
            }
#pragma unroll
            for (int j = 0; j < kDenseBatch; ++j) {
                a0 = fma(x0[j].x, fv[j].x, a0);
                a1 = fma(x0[j].y, fv[j].y, a1);
                b0 = fma(x1[j].x, fv[j].x, b0);
                b1 = fma(x1[j].y, fv[j].y, b1);
            }
        }
    } else {   // the last (partial) segment: one column per lane per step
        for (int64_t c = c0 + lane; c < cend; c += 64) {
            const double fv = f[c];
            a0 = fma(m0[c], fv, a0);
            b0 = fma(m1[c], fv, b0);
        }
    }
    const double s0 = wave_total(a0 + a1), s1 = wave_total(b0 + b1);   // uniform across the wave
    if (nseg == 1) {
        if (lane == 0) {
            if (r0 < n) y[r0] = ADD ? add[r0] + s0 : s0;
            if (r1 < n) y[r1] = ADD ? add[r1] + s1 : s1;
        }
        return;
    }
    // split rows: each unit publishes its two row partials into slots armed with the gridsum sentinel
    // (agent-scope stores, value-is-flag: no fence, which on gfx950 would write back the whole L2 per
    // workgroup), then draws a ticket on its row block's counter; the holder of the last ticket sums the
    // nseg partials of each row in segment order (every other unit's stores were issued before its ticket,
    // so each poll ends), re-arms the slots and resets the counter (psk_internal.hpp "gridsum" protocol).
    if (lane == 0) {
        if (r0 < n) gridsum_put(part + (int64_t)seg * n + r0, s0);
        if (r1 < n) gridsum_put(part + (int64_t)seg * n + r1, s1);
    }
    __syncthreads();
    __shared__ uint32_t tk;
    if (threadIdx.x == 0) tk = gridsum_draw(cnt + rb * kDenseCntStride);
    __syncthreads();
    if (tk != (uint32_t)nseg - 1) return;   // not the row block's last unit
    if (threadIdx.x == 0) gridsum_reset(cnt + rb * kDenseCntStride);
    const int64_t r = rb * kDenseRows + threadIdx.x;
    if (threadIdx.x < kDenseRows && r < n) {
        double s = 0.0;
        for (int32_t q = 0; q < nseg; ++q) {
            uint64_t *sl = part + (int64_t)q * n + r;
            s += __longlong_as_double((long long)gridsum_wait(sl, err));
            __hip_atomic_store(sl, kGridSumSentinel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        y[r] = ADD ? add[r] + s : s;
    }
}

__global__ void dense_arm_kernel(int64_t m, uint64_t *part) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) part[i] = kGridSumSentinel;
}

static int dense_gemv(const DenseInverse *d, int64_t n, const double *f, const double *add, double *y,
                      hipStream_t s) {
    const dim3 grid((unsigned)(d->nrb * d->nseg));
    if (add)
        hipLaunchKernelGGL(dense_gemv_kernel<true>, grid, dim3(kBlock), 0, s, n, d->ld, d->nseg, d->M, f, add, y,
                           d->part, d->cnt, d->err);
    else
        hipLaunchKernelGGL(dense_gemv_kernel<false>, grid, dim3(kBlock), 0, s, n, d->ld, d->nseg, d->M, f, add,
                           y, d->part, d->cnt, d->err);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

int dense_apply(const psk_prec *P, const double *v, double *out, hipStream_t s) {
    const DenseInverse *d = P->dense;
    const int64_t n = P->n;
    if (((uintptr_t)v & 15) != 0)
        return fail(PSK_ERR_ARG, "dense inverse apply: the input vector must be 16-byte aligned");
    if (d->refine == 0) return dense_gemv(d, n, v, nullptr, out, s);
    double *x1 = d->work, *r = d->work + d->ld;   // (r 16-byte aligned: ld is a multiple of 8)
    PSK_TRY(dense_gemv(d, n, v, nullptr, x1, s));
    for (int it = 0; it < d->refine; ++it) {   // x <- x + A^-1 (f - A x)
        PSK_TRY(launch_spmv(d->A, kSpmvResid, x1, r, nullptr, v, nullptr, nullptr, s));
        double *dst = it + 1 == d->refine ? out : x1;
        PSK_TRY(dense_gemv(d, n, r, x1, dst, s));   // (dst may alias add: each y[i] reads add[i] first)
    }
    return PSK_OK;
}

int dense_check_error(const psk_prec *P, hipStream_t s) {
    const DenseInverse *d = P->dense;
    if (!d || !d->err) return PSK_OK;
    int32_t h = 0;
    PSK_HIP(hipMemcpyAsync(&h, d->err, 4, hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    if (h) {
        (void)hipMemsetAsync(d->err, 0, sizeof(int32_t), s);
        (void)hipStreamSynchronize(s);
        return fail(PSK_ERR_HIP, "dense inverse apply: a partial sum never landed (bounded wait expired)");
    }
    return PSK_OK;
}

// ---------------------------------------------------------------------------------------------
// rocSOLVER, resolved at first use: the library is ~0.9 GB and only the dense coarse solve needs it
namespace {
typedef int rb_status;   // rocblas_status
typedef void *rb_handle;
struct Rocsolver {
    rb_status (*create)(rb_handle *) = nullptr;
    rb_status (*destroy)(rb_handle) = nullptr;
    rb_status (*set_stream)(rb_handle, hipStream_t) = nullptr;
    rb_status (*getrf)(rb_handle, int32_t, int32_t, double *, int32_t, int32_t *, int32_t *) = nullptr;
    rb_status (*getri)(rb_handle, int32_t, double *, int32_t, int32_t *, int32_t *) = nullptr;
    std::string err;
};
const Rocsolver &rocsolver() {
    static Rocsolver r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            r.err = std::string("dlopen librocsolver: ") + (e ? e : "?");
            return;
        }
        r.create = (rb_status(*)(rb_handle *))dlsym(h, "rocblas_create_handle");
        r.destroy = (rb_status(*)(rb_handle))dlsym(h, "rocblas_destroy_handle");
        r.set_stream = (rb_status(*)(rb_handle, hipStream_t))dlsym(h, "rocblas_set_stream");
        r.getrf = (rb_status(*)(rb_handle, int32_t, int32_t, double *, int32_t, int32_t *, int32_t *))dlsym(
            h, "rocsolver_dgetrf");
        r.getri = (rb_status(*)(rb_handle, int32_t, double *, int32_t, int32_t *, int32_t *))dlsym(
            h, "rocsolver_dgetri");
        if (!r.create || !r.destroy || !r.set_stream || !r.getrf || !r.getri) r.err = "rocSOLVER symbols missing";
    });
    return r;
}
}  // namespace

}  // namespace psk

using namespace psk;

extern "C" int psk_prec_create_dense_inverse(const psk_csr *A, int32_t refine, psk_prec **out) {
    if (!A || !out || refine < 0 || refine > 4) return fail(PSK_ERR_ARG, "psk_prec_create_dense_inverse: bad arguments");
    if (A->comm) return fail(PSK_ERR_UNSUPPORTED, "psk_prec_create_dense_inverse: sharded matrix");
    if (A->ncols != A->n) return fail(PSK_ERR_ARG, "psk_prec_create_dense_inverse: matrix not square");
    const int64_t n = A->n;
    const int64_t ld = (n + 7) / 8 * 8;
    if (n > kDenseMaxN) return fail(PSK_ERR_UNSUPPORTED, "psk_prec_create_dense_inverse: n above the dense limit");
    Context *c;
    PSK_TRY(ctx(&c));
    DenseInverse *d = new DenseInverse();
    d->ld = ld;
    d->A = A;
    d->refine = refine;
    d->nseg = (int32_t)std::max<int64_t>(1, (n + kDenseCols - 1) / kDenseCols);
    d->nrb = (n + kDenseRows - 1) / kDenseRows;
    auto bail = [&](int code, const std::string &m) {
        dense_free(d);
        return fail(code, "psk_prec_create_dense_inverse: " + m);
    };
    psk_prec *P = new psk_prec();
    P->kind = PSK_PREC_DENSE;
    P->n = n;
    if (n == 0) {
        P->dense = d;
        *out = P;
        return PSK_OK;
    }
    // a failed hipMalloc leaves HIP's sticky error set: cleared here, so the caller's fallback (AMG auto mode: the
    // SuperLU factors) does not read it as its own launch error
    auto alloc = [&](void **p, size_t bytes) {
        if (hipMalloc(p, bytes) == hipSuccess) return true;
        *p = nullptr;
        (void)hipGetLastError();
        return false;
    };
    {   // never more than half of what the device has free (the inverse is 8 n^2 bytes, allocated silently)
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
            (void)hipGetLastError();
            fr = 0;
        }
        if ((double)n * ld * 8.0 > 0.5 * (double)fr) {
            delete P;
            return bail(PSK_ERR_ALLOC, "the " + std::to_string((double)n * ld * 8 / 1e9) +
                                           " GB inverse exceeds half of the free device memory");
        }
    }
    if (!alloc((void **)&d->M, (size_t)n * ld * sizeof(double)) ||
        (d->nseg > 1 && !alloc((void **)&d->part, (size_t)d->nseg * n * sizeof(uint64_t))) ||
        (d->nseg > 1 && !alloc((void **)&d->cnt, (size_t)d->nrb * kDenseCntStride * sizeof(uint32_t))) ||
        !alloc((void **)&d->err, sizeof(int32_t)) ||
        (refine > 0 && !alloc((void **)&d->work, (size_t)2 * ld * sizeof(double)))) {
        delete P;
        return bail(PSK_ERR_ALLOC, "hipMalloc (" + std::to_string((double)n * ld * 8 / 1e9) + " GB inverse)");
    }
    int32_t *ipiv = nullptr, *info = nullptr;
    if (!alloc((void **)&ipiv, (size_t)n * sizeof(int32_t)) || !alloc((void **)&info, 2 * sizeof(int32_t))) {
        if (ipiv) (void)hipFree(ipiv);
        delete P;
        return bail(PSK_ERR_ALLOC, "hipMalloc pivots");
    }
    auto done = [&](int code, const std::string &m) {
        (void)hipFree(ipiv);
        (void)hipFree(info);
        if (code == PSK_OK) return PSK_OK;
        delete P;
        return bail(code, m);
    };
    hipStream_t s = c->stream;
    hipError_t e = hipMemsetAsync(d->M, 0, (size_t)n * ld * sizeof(double), s);
    if (e == hipSuccess && d->cnt) e = hipMemsetAsync(d->cnt, 0, (size_t)d->nrb * kDenseCntStride * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(d->err, 0, sizeof(int32_t), s);
    if (e == hipSuccess && d->part) {
        const int64_t m = (int64_t)d->nseg * n;
        hipLaunchKernelGGL(dense_arm_kernel, dim3((unsigned)((m + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, m, d->part);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemsetAsync(info, 0, 2 * sizeof(int32_t), s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(dense_scatter_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n,
                           ld, A->rowptr, A->colidx, A->vals, d->M);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return done(PSK_ERR_HIP, std::string("scatter: ") + hipGetErrorString(e));
    const Rocsolver &rs = rocsolver();
    if (!rs.err.empty()) return done(PSK_ERR_UNSUPPORTED, rs.err);
    rb_handle h = nullptr;
    // rocBLAS/rocSOLVER failures are reported as unsupported, so auto mode falls back to the factors
    if (rs.create(&h) != 0) return done(PSK_ERR_UNSUPPORTED, "rocblas_create_handle");
    int st = rs.set_stream(h, s);
    // column-major view of the row-major image: A^T; its inverse read row-major is A^-1
    if (st == 0) st = rs.getrf(h, (int32_t)n, (int32_t)n, d->M, (int32_t)ld, ipiv, info);
    if (st == 0) st = rs.getri(h, (int32_t)n, d->M, (int32_t)ld, ipiv, info + 1);
    int32_t hinfo[2] = {0, 0};
    e = hipMemcpyAsync(hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    rs.destroy(h);
    if (st != 0) return done(PSK_ERR_UNSUPPORTED, "rocSOLVER getrf/getri status " + std::to_string(st));
    if (e != hipSuccess) return done(PSK_ERR_HIP, hipGetErrorString(e));
    if (hinfo[0] != 0 || hinfo[1] != 0)
        return done(PSK_ERR_ARG, "singular matrix (getrf info " + std::to_string(hinfo[0]) + ", getri info " +
                                     std::to_string(hinfo[1]) + ")");
    P->dense = d;
    *out = P;
    return done(PSK_OK, "");
}
