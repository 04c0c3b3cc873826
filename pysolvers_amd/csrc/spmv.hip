// spmv.hip — CSR SpMV (the hot kernel), the CSR handle, the FD generator, Jacobi, BLAS-1 entry points.
//
// SpMV replaces mvmult(A, x) (IterativeLinearSolver.py:94-106) = scipy csr_matvec: for each row,
// sum = 0; sum += vals[jj] * x[colidx[jj]] in STORED order, product rounded before the add.
// We reproduce that bit for bit: the products are staged through LDS (so no FMA can form) and each
// row is summed sequentially by one lane in stored order, starting from 0.0.
//
// Layout/schedule (gfx950): one workgroup of 256 threads (4 waves) per tile of `trows` rows (256
// for 5-point rows), grid = tiles (one-shot; see gridsum in psk_internal.hpp for why). The tile's
// nnz range [rowptr[r0], rowptr[r1]) is streamed in 1280-entry chunks with fully coalesced
// non-temporal loads of colidx (4 B/lane) and vals (8 B/lane), the x gather is issued branch-free
// for 5 entries per lane, rounded products land in a 10 KiB LDS slab, and each lane then sums its
// own row from LDS. Rows longer than a chunk keep their running sum across chunks, so ANY row
// length is exact. Optional epilogues fuse the dot products the Krylov loops need next (p.Ap for
// PCG, q_0.u for GMRES, ||b-Ax||^2 for the true residual), reduced deterministically by gridsum.
#include "psk_internal.hpp"
#include "pcg_state.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cmath>

namespace psk {

// Stream loads of colidx/vals (read once per SpMV) are non-temporal; the x gathers keep the default
// policy so neighbouring grid lines are served from L2 / Infinity Cache (tools/spmv_lab.hip A/B:
// nt on the stream +9-12% at n = 10M / 16.7M).
__device__ __forceinline__ int32_t ld_stream(const int32_t *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ double ld_stream(const double *p) { return __builtin_nontemporal_load(p); }

// The dot epilogue of every SpMV kernel (p.Ap, q_0.u, ||b-Ax||^2): one DPP total per WAVE, the
// tile's wave totals added in LDS in wave order and published as one gridsum slot per tile
// (gridsum_tile_*, psk_internal.hpp) — no workgroup barrier at the end of a slice. Both layouts sum
// 64 rows per wave in the same lanes over the same 256-row tiles, so their grid sums are
// bit-identical.
template <int MODE>
__device__ __forceinline__ bool spmv_publishes(const GridSum &gs) {
    return MODE != kSpmvPlain && MODE != kSpmvAdd && (MODE != kSpmvResid || gs.out != nullptr);
}
template <int MODE>
__device__ __forceinline__ uint32_t spmv_begin(const GridSum &gs, GridSumTile<1> &L, int64_t t) {
    return spmv_publishes<MODE>(gs) ? gridsum_tile_begin<1>(gs, L, t) : 0u;
}
__device__ __forceinline__ void spmv_publish(const GridSum &gs, GridSumTile<1> &L, double acc, uint32_t ticket,
                                             int64_t t) {
    const double ws = wave_total(acc);
    gridsum_tile_publish<1>(gs, L, &ws, ticket, t);
}

// The row's y value and dot partial first, the y store after the
// dot epilogue (gridsum publish). On gfx950 the registers holding a store's data may not be reused
// until the store has left (a vmcnt wait that also waits for its HBM write): with the y store ahead
// of the epilogue, every wave waited for it there (kSpmvDot at N = 10M: ~9.5 us over a plain SpMV).
template <int MODE>
__device__ __forceinline__ double spmv_row_value(bool has, double sum, double eq, double &acc) {
    const double yv = MODE == kSpmvResid ? eq - sum : MODE == kSpmvAdd ? eq + sum : sum;   // :163 / VCycleManager.py:55
    acc = 0.0;
    if (has && MODE != kSpmvPlain && MODE != kSpmvAdd) acc = MODE == kSpmvResid ? yv * yv : eq * sum;
    return yv;
}
template <int MODE>
__device__ __forceinline__ void spmv_store_row(bool has, int64_t row, double yv, double *__restrict__ y) {
    if (!has) return;
    if (MODE == kSpmvResid || MODE == kSpmvAdd) y[row] = yv;
    else __builtin_nontemporal_store(yv, y + row);
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void spmv_kernel(
    int64_t n, int trows, const int32_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const double *__restrict__ vals, const double *__restrict__ x, double *__restrict__ y,
    const double *__restrict__ aux_d, const double *__restrict__ aux_q, GridSum gs,
    const int32_t *__restrict__ done, int32_t nnz, TileMap tm) {
    if (done != nullptr && *done != 0) return;
    constexpr int KU = kChunk / kBlock;   // staged entries per lane per chunk
    __shared__ double prod[kChunk + kBlock];   // + a dump row for lanes past the chunk's end
    const int tid = threadIdx.x;
    const int64_t t = tile_of_block(tm);
    const int64_t r0 = t * trows;
    const int64_t r1 = (r0 + trows < n) ? r0 + trows : n;
    const int32_t last = nnz > 0 ? nnz - 1 : 0;   // colidx/vals hold at least one (dummy) entry
    const int32_t e0 = rowptr[r0], e1 = rowptr[r1];
    // the first chunk's colidx/vals stream, clamped to valid indices (an empty tile re-reads one
    // valid entry), issued before anything else
    int32_t cc[KU];
    double vv[KU];
    {
        const int32_t c1 = (e1 - e0 > kChunk) ? e0 + kChunk : e1;
        const int32_t base = e0 < last ? e0 : last;
#pragma unroll
        for (int k = 0; k < KU; ++k) {
            const int32_t e = e0 + k * kBlock + tid;
            const int32_t ee = e < c1 ? e : base;
            cc[k] = ld_stream(colidx + ee);
            vv[k] = ld_stream(vals + ee);
        }
    }
    __shared__ GridSumTile<1> gsl;
    const uint32_t ticket = spmv_begin<MODE>(gs, gsl, t);
    const int64_t row = r0 + tid;
    const bool has = tid < trows && row < r1;
    const int64_t rowc = has ? row : r0;   // a valid row for the unconditional epilogue loads
    const int32_t rs = rowptr[rowc], re = rowptr[rowc + 1];
    double eq = 0.0;
    if (MODE == kSpmvDot) eq = x[rowc];
    if (MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot)
        eq = aux_q[rowc];
    double sum = 0.0;
    {   // chunk 0
        const int32_t c0 = e0, c1 = (e1 - c0 > kChunk) ? c0 + kChunk : e1;
        double pv[KU];
#pragma unroll
        for (int k = 0; k < KU; ++k) {
            double xx = x[cc[k]];
            if (MODE == kSpmvJacobiDot) xx = aux_d[cc[k]] * xx;   // (DInv*q)[c], rounded
            pv[k] = vv[k] * xx;                                   // rounded product
        }
#pragma unroll
        for (int k = 0; k < KU; ++k) {   // lanes past the chunk write the dump row
            const int32_t e = c0 + k * kBlock + tid;
            prod[(e < c1 ? k * kBlock : kChunk) + tid] = pv[k];
        }
        __syncthreads();
        const int32_t a = rs > c0 ? rs : c0;
        const int32_t bnd = re < c1 ? re : c1;
        if (has)
            for (int32_t e = a; e < bnd; ++e) sum = sum + prod[e - c0];   // stored order
        __syncthreads();
    }
    // rare: tile longer than one chunk
    for (int32_t c0 = e0 + kChunk; c0 < e1; c0 += kChunk) {
        const int32_t c1 = (e1 - c0 > kChunk) ? c0 + kChunk : e1;
        double pv[KU];
#pragma unroll
        for (int k = 0; k < KU; ++k) {
            const int32_t e = c0 + k * kBlock + tid;
            const int32_t ee = e < c1 ? e : c0;
            const int32_t c = ld_stream(colidx + ee);
            double xx = x[c];
            if (MODE == kSpmvJacobiDot) xx = aux_d[c] * xx;
            pv[k] = ld_stream(vals + ee) * xx;
        }
#pragma unroll
        for (int k = 0; k < KU; ++k) {
            const int32_t e = c0 + k * kBlock + tid;
            if (e < c1) prod[k * kBlock + tid] = pv[k];
        }
        __syncthreads();
        const int32_t a = rs > c0 ? rs : c0;
        const int32_t bnd = re < c1 ? re : c1;
        if (has)
            for (int32_t e = a; e < bnd; ++e) sum = sum + prod[e - c0];
        __syncthreads();
    }
    double acc;
    const double yv = spmv_row_value<MODE>(has, sum, eq, acc);
    // only the residual mode may be called without partials (AMG smoothing); kernel-uniform test
    if (spmv_publishes<MODE>(gs)) spmv_publish(gs, gsl, acc, ticket, t);
    spmv_store_row<MODE>(has, row, yv, y);
}

// ---------------------------------------------------------------------------------------------
// Sliced layout (SELL-256): the same entries regrouped so that one workgroup owns a slice of
// kSlice = 256 rows, ONE ROW PER LANE, and slot j of the slice's rows is contiguous (slot-major).
// The stream loads stay coalesced, and each x gather instruction of a wave now reads the j-th
// entries of 64 consecutive rows: for the 5-point matrix 512 contiguous bytes of x per slot, where
// a CSR tile's gather instruction mixes the 5 neighbour offsets of ~13 rows (more cache lines and
// address work per load). Each lane still sums ITS row in stored order from 0.0 with rounded
// products, so y is bit-identical to csr_matvec and to spmv_kernel. Padding slots (rows shorter
// than the slice's widest row) are skipped. No rowptr stream, no LDS staging.
// Storage of a slice of width w (slot offset o = sl_off[t], all arrays indexed from o):
//  * values in slot PAIRS: slots 2p, 2p+1 of lane l adjacent at o + 2p*256 + 2l (one 16-B load per
//    pair); an odd last slot at o + (w-1)*256 + l;
//  * columns, by sl_fmt[t]: a "packed" slice (every column within +-32767 of its row) stores the
//    int16 deltas c - row of slots 2p, 2p+1 in ONE int32 word at word wo + p*256 + l of the word
//    stream sl_pcol (wo = sl_woff[t]; kPad16 = padding), i.e. 2 B per slot in full 256-B wave
//    loads; any other slice int32 columns at o + j*256 + l of sl_col (-1 = padding). FD: 10.4 B per
//    slot instead of 12 (every slice but a shard's halo lines).
//  * values, when the whole matrix holds at most kDictMax distinct values (bit patterns; stencils,
//    graph Laplacians, FEM on uniform meshes): a value DICTIONARY (sl_dict) and one byte per slot,
//    the indices of slots 4q..4q+3 of lane l in one 32-bit word of the word stream, after the
//    slice's column words (word wo + ceil(w/2)*256 + q*256 + l; wo + q*256 + l in a wide slice), so
//    a slice's whole stream is one contiguous run; 3 B per slot with packed columns instead of 10
//    (no sl_val then). The kernel keeps the dictionary in scalar registers and picks a
//    slot's value with a select tree (no memory instruction per slot: tools/dict_lab.hip, FD
//    16384^2: doubles 2.96 ms, indices + dict[idx] loads 2.24 ms, indices + selects 1.70 ms). The
//    dictionary entries are the matrix's own doubles, so every product, and y, is unchanged bit for
//    bit (Kourtis et al., "CSR-VI" value compression).
// tools/sell_lab.hip, tools/sell_pack_lab.hip (16384^2, back to back): CSR 3.61 ms, int32 columns
// 3.20-3.39 ms, 16-bit pairs + paired values 2.87 ms; all bit-identical.
constexpr int kSlice = kBlock;
constexpr int kDictMax = 8;      // distinct values a dictionary may hold (held in scalar registers)
constexpr int kDictCand = 64;    // candidates one detection pass collects
constexpr int kSliceRegs = 8;             // slots held in registers; wider slices take the loop below
constexpr int16_t kPad16 = INT16_MIN;     // padding slot of a packed slice
constexpr int64_t kMaxDelta16 = 32767;

// value of slot j (of w) of lane l in a slice at slot offset o
__device__ __forceinline__ int64_t sliced_vpos(int64_t o, int j, int w, int l) {
    return (j | 1) < w ? o + (int64_t)(j & ~1) * kSlice + 2 * l + (j & 1) : o + (int64_t)j * kSlice + l;
}

__device__ __forceinline__ int32_t unpack_delta(int32_t row, int16_t d) { return d == kPad16 ? -1 : row + (int32_t)d; }

__device__ __forceinline__ bool same_bits(double a, double b) {
    return __double_as_longlong(a) == __double_as_longlong(b);
}

// the dictionary as named scalars (an array here was promoted to per-thread LDS copies)
struct DictRegs {
    double d0, d1, d2, d3, d4, d5, d6, d7;
};

// dictionary entry idx (< DK) by selects on the index bits; the entries live in scalar registers
template <int DK>
__device__ __forceinline__ double dict_pick(const DictRegs dv, uint32_t idx) {
    if (DK == 2) return (idx & 1) ? dv.d1 : dv.d0;
    const double a0 = (idx & 1) ? dv.d1 : dv.d0, a1 = (idx & 1) ? dv.d3 : dv.d2;
    const double b0 = (idx & 2) ? a1 : a0;
    if (DK == 4) return b0;
    const double a2 = (idx & 1) ? dv.d5 : dv.d4, a3 = (idx & 1) ? dv.d7 : dv.d6;
    const double b1 = (idx & 2) ? a3 : a2;
    return (idx & 4) ? b1 : b0;
}

// a done flag that is never set, for launches without one (the kernel reads the flag without a
// branch on the pointer, so its load goes out with the slice header)
__device__ int32_t g_spmv_never_done = 0;

#ifdef PSK_SPMV_PROF
// development probe (tools/spmv_probe.py, a -DPSK_SPMV_PROF build): s_memrealtime (100 MHz, one clock for
// every XCD) per workgroup of the last launch: [0] entry, [1] sums done (before the dot epilogue), [2] end;
// per group reduction [start, end] at kSpmvProfGrp + 2g, the final reduction at kSpmvProfFin
constexpr int kSpmvProfWg = 32768, kSpmvProfGrp = 3 * kSpmvProfWg, kSpmvProfFin = kSpmvProfGrp + 2 * 4096;
__device__ unsigned long long g_spmv_prof[kSpmvProfFin + 2];
extern "C" int psk_spmv_prof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spmv_prof), sizeof(g_spmv_prof)) == hipSuccess ? 0 : -1;
}
#define PSK_SPMV_PROF_AT(slot) \
    do { if (threadIdx.x == 0 && blockIdx.x < kSpmvProfWg) g_spmv_prof[blockIdx.x * 3 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PSK_SPMV_PROF_AT(slot) do { } while (0)
#endif

// The dictionary entries DK needs, as scalar loads (the buffer is padded to kDictMax entries).
template <int DK>
__device__ __forceinline__ DictRegs load_dict(const double *__restrict__ sdict) {
    DictRegs dv{};
    if (DK >= 2) {
        dv.d0 = sdict[0];
        dv.d1 = sdict[1];
    }
    if (DK >= 4) {
        dv.d2 = sdict[2];
        dv.d3 = sdict[3];
    }
    if (DK >= 8) {
        dv.d4 = sdict[4];
        dv.d5 = sdict[5];
        dv.d6 = sdict[6];
        dv.d7 = sdict[7];
    }
    return dv;
}

// x[row] for the PCG dot p.Ap (kSpmvDot): the gathered value of the row's diagonal slot when it
// stores one (every 5-point row does: x[c] with c == row is the same double), else a load (rare:
// the branch is taken by the lanes whose row has no stored diagonal). Loading x[row] up front with
// the stream cost 7% of the in-loop SpMV at FD 16384^2 (one more load in the first round trip).
template <int NS>
__device__ __forceinline__ double diag_x(const int32_t *cc, const double *xv, int32_t row, const double *__restrict__ x,
                                         bool has) {
    double d = 0.0;
    bool found = false;
#pragma unroll
    for (int j = 0; j < NS; ++j)
        if (cc[j] == row) {
            d = xv[j];
            found = true;
        }
    if (!found && has) d = x[row];
    return d;
}

// Uniform layout (every slice UW wide and packed — FD and other constant-width banded matrices):
// the width is a template parameter, so the slice's whole stream is issued as one batch of
// unconditional loads (a runtime width put a branch between consecutive loads and the compiler
// then waited on each one: four memory round trips per slice instead of two), the offsets are
// computed from the slice index, and every slot's gather is issued unconditionally (padding slots
// gather x[0], and their product is skipped). DK: dictionary size class (0 = double values in slot
// pairs, 2 / 4 / 8 entries). CMP (odd UW, DK = 2): entry j's 1-bit value index is bit j of the last
// column word's upper half — the half an odd width leaves unused — so no index words are streamed
// (FD: 12 instead of 20 B/row of stream).
template <int MODE, int DK, int UW, bool CMP = false>
__global__ __launch_bounds__(kBlock) void spmv_uniform_kernel(
    int64_t n, const int32_t *__restrict__ spcol, const double *__restrict__ sval, const double *__restrict__ sdict,
    const double *__restrict__ x, double *__restrict__ y, const double *__restrict__ aux_d,
    const double *__restrict__ aux_q, GridSum gs, const int32_t *__restrict__ done, TileMap tm) {
    constexpr int NP = (UW + 1) / 2;                 // packed column words per lane
    static_assert(!CMP || (DK == 2 && (UW & 1)), "compact stream: odd width, 2-entry dictionary");
    constexpr int NI = DK > 0 && !CMP ? (UW + 3) / 4 : 0;   // dictionary index words per lane
    const int32_t dn = *(done ? done : &g_spmv_never_done);   // tested once the stream is in flight
    const int tid = threadIdx.x;
    const int64_t t = tile_of_block(tm), row = t * kSlice + tid;
    const bool has = row < n;
    const int32_t *pword = spcol + t * (int64_t)((NP + NI) * kSlice) + tid;
    uint32_t cw[NP], iw[NI > 0 ? NI : 1];
    double vv[UW];
#pragma unroll
    for (int p = 0; p < NP; ++p) cw[p] = (uint32_t)ld_stream(pword + p * kSlice);
    if (DK > 0) {
#pragma unroll
        for (int q = 0; q < NI; ++q) iw[q] = (uint32_t)ld_stream(pword + (NP + q) * kSlice);
        if (CMP) iw[0] = 0;
    } else {
        const double *v0 = sval + t * (int64_t)(UW * kSlice);
#pragma unroll
        for (int p = 0; p < UW / 2; ++p) {
            const dv2 v2 = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(v0 + 2 * p * kSlice) + tid);
            vv[2 * p] = v2.x;
            vv[2 * p + 1] = v2.y;
        }
        if (UW & 1) vv[UW - 1] = ld_stream(v0 + (UW - 1) * kSlice + tid);
    }
    const int64_t rowc = has ? row : 0;
    double eq = 0.0;
    // kSpmvDot's x[row] is not loaded here: a row that stores its diagonal gathers it below
    if (MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot) eq = aux_q[rowc];
    const DictRegs dv = load_dict<DK>(sdict);
    if (dn != 0) {   // uniform over the launch: no barrier has been passed
        // the stream loads are consumed on this path too, so the compiler issues them ahead of the
        // test instead of sinking them below it (every slice would wait on the flag first)
#pragma unroll
        for (int p = 0; p < NP; ++p) __asm__ volatile("" ::"v"(cw[p]));
        if (DK > 0) {
#pragma unroll
            for (int q = 0; q < NI; ++q) __asm__ volatile("" ::"v"(iw[q]));
        } else {
#pragma unroll
            for (int j = 0; j < UW; ++j) __asm__ volatile("" ::"v"(vv[j]));
        }
        return;
    }
    __shared__ GridSumTile<1> gsl;
    const uint32_t ticket = spmv_begin<MODE>(gs, gsl, t);
    const int32_t row32 = (int32_t)row;
    int32_t cc[UW];
    double xv[UW];
#pragma unroll
    for (int j = 0; j < UW; ++j) {
        cc[j] = unpack_delta(row32, (int16_t)((j & 1) ? (cw[j >> 1] >> 16) : (cw[j >> 1] & 0xffff)));
        const int32_t cl = cc[j] >= 0 ? cc[j] : 0;
        xv[j] = x[cl];
        if (MODE == kSpmvJacobiDot) xv[j] = aux_d[cl] * xv[j];   // (DInv*q)[c], rounded
    }
    if (DK > 0) {
#pragma unroll
        for (int j = 0; j < UW; ++j)
            vv[j] = dict_pick<DK>(dv, CMP ? (cw[NP - 1] >> (16 + j)) & 1u : (iw[j >> 2] >> (8 * (j & 3))) & 0xff);
    }
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < UW; ++j)
        if (cc[j] >= 0) sum = sum + vv[j] * xv[j];   // stored order, rounded product
    if (MODE == kSpmvDot) eq = diag_x<UW>(cc, xv, row32, x, has);
    double acc;
    const double yv = spmv_row_value<MODE>(has, sum, eq, acc);
    if (spmv_publishes<MODE>(gs)) spmv_publish(gs, gsl, acc, ticket, t);
    spmv_store_row<MODE>(has, row, yv, y);
}

// The dot epilogue of a workgroup holding TPW gridsum tiles: first every tile's slot is combined in LDS
// and stored (no wait of any kind), only then does a wave that published a tile holding its group's
// last ticket reduce that group. Storing every slot before any reduction keeps the protocol's
// guarantee: a reducer only waits on tiles that drew their tickets earlier, and those store all their
// slots without waiting — a wave reducing tile 0's group while tile 1's slot were still unstored could
// otherwise close a cycle of reducers across workgroups.
template <int TPW>
__device__ __forceinline__ void spmv_publish_multi(const GridSum &gs, GridSumTile<1> *L, const double *acc,
                                                   const uint32_t *ticket, const int64_t *tl, const bool *tv) {
    const bool lane0 = (threadIdx.x & 63) == 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    bool mine[TPW];
    uint32_t tk[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        mine[q] = false;
        tk[q] = 0;
        if (!tv[q]) continue;   // uniform: the last workgroup's missing slice
        const double ws = wave_total(acc[q]);
        uint32_t old = 0;
        if (lane0) {
            L[q].part[wave] = ws;
            if (threadIdx.x == 0) L[q].ticket = ticket[q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            old = atomicAdd(&L[q].cnt, 1u);
        }
        if (__builtin_amdgcn_readfirstlane(old) != kWaves - 1) continue;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        double sum = L[q].part[0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) sum += L[q].part[w];   // wave order
        tk[q] = L[q].ticket;
        if (lane0)
            gridsum_put(gs.grp_log2 < 0 ? gs.gslots + tl[q] : gs.slots + gridsum_slot(gs, tl[q]), sum);
        mine[q] = true;
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        if (!mine[q]) continue;
        if (gs.grp_log2 < 0) {
            gridsum_final_wave<1>(gs);
            continue;
        }
        const int64_t g = gridsum_group_of(tl[q], gs.grp_log2);
        int64_t base;
        const int64_t cnt = gridsum_members(gs, g, base);
        if (tk[q] != (uint32_t)(cnt - 1)) continue;
#ifdef PSK_SPMV_PROF
        if (lane0 && g < 4096) g_spmv_prof[kSpmvProfGrp + 2 * g] = __builtin_amdgcn_s_memrealtime();
#endif
        double r[1];
        gridsum_take<1, 64>(gs.slots, g << gs.grp_log2, cnt, gs.err, nullptr, r);
        if (lane0) {
            gridsum_reset(gridsum_counter(gs, g));
            gridsum_put(gs.gslots + g, r[0]);
        }
#ifdef PSK_SPMV_PROF
        if (lane0 && g < 4096) g_spmv_prof[kSpmvProfGrp + 2 * g + 1] = __builtin_amdgcn_s_memrealtime();
        const uint64_t tf = __builtin_amdgcn_s_memrealtime();
#endif
        gridsum_final_wave<1>(gs);
#ifdef PSK_SPMV_PROF
        if (lane0) {
            const uint64_t te = __builtin_amdgcn_s_memrealtime();
            if (te - tf > 20) {   // > 200 ns: this wave ran the final reduction (a non-final return is immediate)
                g_spmv_prof[kSpmvProfFin] = tf;
                g_spmv_prof[kSpmvProfFin + 1] = te;
            }
        }
#endif
    }
}

// The uniform kernel with TPW slices per workgroup, one row of each per lane (rows t*256 + lane of the
// TPW consecutive slices t of the workgroup): every stream load of all TPW slices is issued first, then
// every gather, so a wave keeps TPW times the bytes in flight of the one-slice kernel (the in-loop
// SpMV at N = 10M moves ~24 KiB per CU at once with one slice, below what streaming needs). The grid
// sums stay per 256-row slice (one gridsum tile each, its own ticket and LDS combine), so p.Ap has the
// same bits as the one-slice kernel and the CSR layout.
template <int MODE, int DK, int UW, bool CMP, int TPW>
__global__ __launch_bounds__(kBlock) void spmv_uniform_multi_kernel(
    int64_t n, const int32_t *__restrict__ spcol, const double *__restrict__ sval, const double *__restrict__ sdict,
    const double *__restrict__ x, double *__restrict__ y, const double *__restrict__ aux_d,
    const double *__restrict__ aux_q, GridSum gs, const int32_t *__restrict__ done, TileMap tm, int64_t ntiles) {
    constexpr int NP = (UW + 1) / 2;
    static_assert(!CMP || (DK == 2 && (UW & 1)), "compact stream: odd width, 2-entry dictionary");
    constexpr int NI = DK > 0 && !CMP ? (UW + 3) / 4 : 0;
    const int32_t dn = *(done ? done : &g_spmv_never_done);
    const int tid = threadIdx.x;
    const int64_t grp = tile_of_block(tm);
    int64_t tl[TPW];     // slice of each part (clamped to a valid slice for the loads)
    bool tv[TPW];        // the part is a real slice
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t t = grp * TPW + q;
        tv[q] = t < ntiles;
        tl[q] = tv[q] ? t : ntiles - 1;
    }
    uint32_t cw[TPW][NP], iw[TPW][NI > 0 ? NI : 1];
    double vv[TPW][UW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int32_t *pword = spcol + tl[q] * (int64_t)((NP + NI) * kSlice) + tid;
#pragma unroll
        for (int p = 0; p < NP; ++p) cw[q][p] = (uint32_t)ld_stream(pword + p * kSlice);
        if (DK > 0) {
#pragma unroll
            for (int i = 0; i < NI; ++i) iw[q][i] = (uint32_t)ld_stream(pword + (NP + i) * kSlice);
            if (CMP) iw[q][0] = 0;
        } else {
            const double *v0 = sval + tl[q] * (int64_t)(UW * kSlice);
#pragma unroll
            for (int p = 0; p < UW / 2; ++p) {
                const dv2 v2 = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(v0 + 2 * p * kSlice) + tid);
                vv[q][2 * p] = v2.x;
                vv[q][2 * p + 1] = v2.y;
            }
            if (UW & 1) vv[q][UW - 1] = ld_stream(v0 + (UW - 1) * kSlice + tid);
        }
    }
    double eq[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        eq[q] = 0.0;
        if (MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot)
            eq[q] = aux_q[row < n ? row : 0];
    }
    const DictRegs dv = load_dict<DK>(sdict);
    if (dn != 0) {
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
#pragma unroll
            for (int p = 0; p < NP; ++p) __asm__ volatile("" ::"v"(cw[q][p]));
            if (DK > 0) {
#pragma unroll
                for (int i = 0; i < NI; ++i) __asm__ volatile("" ::"v"(iw[q][i]));
            } else {
#pragma unroll
                for (int j = 0; j < UW; ++j) __asm__ volatile("" ::"v"(vv[q][j]));
            }
        }
        return;
    }
    constexpr bool PUB = MODE != kSpmvPlain && MODE != kSpmvAdd;
    __shared__ GridSumTile<1> gsl[TPW];
    uint32_t ticket[TPW];
    const bool pub = PUB && spmv_publishes<MODE>(gs);
    if (pub) {
        if (tid < TPW) gsl[tid].cnt = 0;
        if (tid == 0 && blockIdx.x == 0 && (gs.nt + TPW - 1) / TPW != gridDim.x) atomicOr(gs.err, 2);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            ticket[q] = 0;
            if (tv[q] && gs.grp_log2 >= 0 && tid == 0)
                ticket[q] = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tl[q], gs.grp_log2)));
        }
    }
    int32_t cc[TPW][UW];
    double xv[TPW][UW], acc[TPW], yv[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int32_t row32 = (int32_t)(tl[q] * kSlice + tid);
#pragma unroll
        for (int j = 0; j < UW; ++j) {
            cc[q][j] = unpack_delta(row32, (int16_t)((j & 1) ? (cw[q][j >> 1] >> 16) : (cw[q][j >> 1] & 0xffff)));
            const int32_t cl = cc[q][j] >= 0 ? cc[q][j] : 0;
            xv[q][j] = x[cl];
            if (MODE == kSpmvJacobiDot) xv[q][j] = aux_d[cl] * xv[q][j];
        }
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        const bool has = tv[q] && row < n;
        if (DK > 0) {
#pragma unroll
            for (int j = 0; j < UW; ++j)
                vv[q][j] = dict_pick<DK>(dv, CMP ? (cw[q][NP - 1] >> (16 + j)) & 1u : (iw[q][j >> 2] >> (8 * (j & 3))) & 0xff);
        }
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < UW; ++j)
            if (cc[q][j] >= 0) sum = sum + vv[q][j] * xv[q][j];   // stored order, rounded product
        if (MODE == kSpmvDot) eq[q] = diag_x<UW>(cc[q], xv[q], (int32_t)row, x, has);
        // y stored after the dot epilogue (spmv_row_value)
        yv[q] = spmv_row_value<MODE>(has, sum, eq[q], acc[q]);
    }
    if (pub) spmv_publish_multi<TPW>(gs, gsl, acc, ticket, tl, tv);
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        spmv_store_row<MODE>(tv[q] && row < n, row, yv[q], y);
    }
}

// ---------------------------------------------------------------------------------------------
// Diagonal layout (round 5; DIA format, Saad's "diagonal storage", with one value per diagonal): when every
// row's entries lie, IN STORED ORDER, on a subsequence of K <= 8 diagonals c = row + d_j, and every entry
// of diagonal j holds the same double v_j (constant-coefficient stencils: FDLaplacian2D's rows are
// [diag, -m, +m, -1, +1] minus the absent neighbours, two distinct values), the whole matrix is the K
// offsets, the K values and ONE presence byte per row (bit j: the row stores an entry on diagonal j).
// Detected at creation (diag_build) by checking every stored entry against the rule, so a row's present
// diagonals, visited in j order, ARE its stored entries in stored order: each lane sums its row from 0.0
// with rounded products exactly as csr_matvec does, and y is bit-identical to the CSR and sliced layouts.
// A row-block shard of such a matrix maps columns outside [0, n) to its halo (c + lo below, c + hi
// above: the FD shard's [owned | halo_lo | halo_hi] columns), checked the same way.
// Stream: 1 B per row instead of the compact sliced layout's 12 (FD at N = 10M: 10 MB instead of 120 MB
// per SpMV); x is gathered and y written as before (16 B per row). Same 256-row slices, one row per lane,
// TPW slices per workgroup and gridsum tiles as spmv_uniform_multi_kernel: p.Ap has the same bits.
constexpr int kDiagMax = 8;
#ifndef PSK_DIAG_TPW
#define PSK_DIAG_TPW 2
#endif
constexpr int kDiagTpw = PSK_DIAG_TPW;   // slices per workgroup
#ifndef PSK_DIAG_DPP
#define PSK_DIAG_DPP 1
#endif
// the -1/+1 diagonals by DPP lane shifts (default from round 5: in-loop SpMV at N = 10M 0.0587 -> 0.0550 ms,
// 16384^2 1.44 -> 1.28 ms, same bits; profiles/r5_diag_dpp_ab.txt; -DPSK_DIAG_DPP=0 builds the gathers)
constexpr bool kDiagDpp = PSK_DIAG_DPP != 0;
struct DiagDesc {
    int32_t d[kDiagMax];   // diagonal offsets, in every row's stored order
    double v[kDiagMax];    // the value (bit pattern) of every entry on diagonal j
    int64_t lo, hi;        // local column of c = row + d: c + lo when c < 0, c + hi when c >= n (shards)
    int64_t ncols;
    int32_t K, jd;         // diagonals; jd = the one with d = 0 (-1: none)
};

__device__ __forceinline__ int64_t diag_col(const DiagDesc &dd, int64_t n, int64_t row, int j) {
    int64_t c = row + dd.d[j];
    c += c < 0 ? dd.lo : (c >= n ? dd.hi : 0);
    return c < 0 ? 0 : (c >= dd.ncols ? dd.ncols - 1 : c);   // absent diagonals gather a valid x (unused)
}

// a zero the compiler cannot see through: turns a uniform load into a per-lane (vector) load
__device__ __forceinline__ int32_t spmv_vzero() {
    int32_t z;
    __asm__ volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

// a double moved one lane along the wave (DPP wavefront shift; both halves by the same pattern): SHR: lane l
// receives lane l-1's value, SHL: lane l+1's; the lane with no source keeps `edge`
template <bool SHR>
__device__ __forceinline__ double wave_shift1(double v, double edge) {
    constexpr int ctrl = SHR ? 0x138 : 0x130;   // wave_shr:1 / wave_shl:1
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// column of row + off under the diagonal layout's mapping (diag_col with an explicit offset)
__device__ __forceinline__ int64_t diag_col_off(const DiagDesc &dd, int64_t n, int64_t row, int64_t off) {
    int64_t c = row + off;
    c += c < 0 ? dd.lo : (c >= n ? dd.hi : 0);
    return c < 0 ? 0 : (c >= dd.ncols ? dd.ncols - 1 : c);
}

// NB (round 5, PSK_DIAG_DPP): the diagonals -1 and +1 are not gathered: lane l's x[row -/+ 1] is
// lane l -/+ 1's x[row] (the d = 0 gather of the same wave), moved by a DPP wave shift; the two wave-edge
// lanes load theirs (one more load instruction, its other lanes re-reading their own x[row]). Exact for
// any mapping: the d = 0 gather of a row r >= n is diag_col(r) = the column of (r - 1) + 1. NB = 1: the
// FD stored order (0, -m, +m, -1, +1); NB = 2: sorted (-m, -1, 0, +1, +m).
template <int MODE, int KM, int TPW, int NB = 0>
__global__ __launch_bounds__(kBlock) void spmv_diag_kernel(
    int64_t n, const uint8_t *__restrict__ mask, DiagDesc dd, const double *__restrict__ x, double *__restrict__ y,
    const double *__restrict__ aux_d, const double *__restrict__ aux_q, GridSum gs, const int32_t *__restrict__ done,
    TileMap tm, int64_t ntiles) {
    constexpr int JD = NB == 1 ? 0 : NB == 2 ? 2 : -1, JM1 = NB == 1 ? 3 : NB == 2 ? 1 : -1,
                  JP1 = NB == 1 ? 4 : NB == 2 ? 3 : -1;
    static_assert(NB == 0 || KM == 5, "NB: the 5-diagonal patterns only");
    PSK_SPMV_PROF_AT(0);
    // ONE memory round trip per workgroup: the done flag (a vector load, so that waiting for it leaves the
    // loads issued after it in flight), the presence bytes and every diagonal's x (clamped addresses that do
    // not depend on the bytes) all go out before anything waits. Tested first, the flag's scalar load and
    // the presence bytes each cost a round trip of their own in front of the gathers (round 5 probe).
    const int32_t dnv = (done ? done : &g_spmv_never_done)[spmv_vzero()];
    const int tid = threadIdx.x;
    const int64_t grp = tile_of_block(tm);
    int64_t tl[TPW];
    bool tv[TPW];
    uint32_t mk[TPW];
    double xv[TPW][KM], eq[TPW], xe[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t t = grp * TPW + q;
        tv[q] = t < ntiles;
        tl[q] = tv[q] ? t : ntiles - 1;
        mk[q] = __builtin_nontemporal_load(mask + tl[q] * kSlice + tid);   // padded to whole slices
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (NB && (j == JM1 || j == JP1)) continue;   // from the d = 0 value of the neighbouring lane
            const int64_t c = diag_col(dd, n, row, j);
            xv[q][j] = x[c];
            if (MODE == kSpmvJacobiDot) xv[q][j] = aux_d[c] * xv[q][j];   // (DInv*q)[c], rounded
        }
        if (NB) {   // the wave-edge lanes' neighbours: lane 0 x[row - 1], lane 63 x[row + 1]
            const int lane = tid & 63;
            const int64_t c = diag_col_off(dd, n, row, lane == 0 ? -1 : (lane == 63 ? 1 : 0));
            xe[q] = x[c];
            if (MODE == kSpmvJacobiDot) xe[q] = aux_d[c] * xe[q];
        }
        eq[q] = 0.0;
        if (MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot)
            eq[q] = aux_q[row < n ? row : 0];
    }
    // the tiles' gridsum tickets drawn now, while the loads are in flight (their values are read at publish)
    constexpr bool PUB = MODE != kSpmvPlain && MODE != kSpmvAdd;
    const bool pub = PUB && spmv_publishes<MODE>(gs);
    uint32_t ticket[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        ticket[q] = 0;
        if (pub && tv[q] && gs.grp_log2 >= 0 && tid == 0)
            ticket[q] = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tl[q], gs.grp_log2)));
    }
    if (__builtin_amdgcn_readfirstlane(dnv) != 0) {   // uniform: the solve has stopped
        // consumed on this path too, so the loads are issued before the test on both; the tickets are
        // handed back (every workgroup of this launch leaves here: nobody reduces)
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            __asm__ volatile("" ::"v"(mk[q]));
            if (NB) __asm__ volatile("" ::"v"(xe[q]));
#pragma unroll
            for (int j = 0; j < KM; ++j)
                if (!(NB && (j == JM1 || j == JP1))) __asm__ volatile("" ::"v"(xv[q][j]));
            if (pub && tv[q] && gs.grp_log2 >= 0 && tid == 0)
                __hip_atomic_fetch_sub(gridsum_counter(gs, gridsum_group_of(tl[q], gs.grp_log2)), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    __shared__ GridSumTile<1> gsl[TPW];
    if (pub) {
        if (tid < TPW) gsl[tid].cnt = 0;
        if (tid == 0 && blockIdx.x == 0 && (gs.nt + TPW - 1) / TPW != gridDim.x) atomicOr(gs.err, 2);
        __syncthreads();
    }
    double acc[TPW], yv[TPW];
    if (NB) {
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            xv[q][JM1] = wave_shift1<true>(xv[q][JD], xe[q]);
            xv[q][JP1] = wave_shift1<false>(xv[q][JD], xe[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        const bool has = tv[q] && row < n;
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < KM; ++j) {   // stored order, rounded product; absent diagonals by a select
            const double t = sum + dd.v[j] * xv[q][j];
            sum = ((mk[q] >> j) & 1u) ? t : sum;
        }
        if (MODE == kSpmvDot) {   // x[row]: the gathered diagonal when the row stores it
            double d = 0.0;
            bool found = false;
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                const bool here = j == dd.jd && ((mk[q] >> j) & 1u);
                d = here ? xv[q][j] : d;
                found = found || here;
            }
            if (!found && has) d = x[row];   // rare: a row without its diagonal
            eq[q] = d;
        }
        yv[q] = spmv_row_value<MODE>(has, sum, eq[q], acc[q]);
    }
#ifdef PSK_SPMV_PROF
    if (threadIdx.x == 0) __asm__ volatile("" ::"v"(acc[0]));
#endif
    PSK_SPMV_PROF_AT(1);
    if (pub) spmv_publish_multi<TPW>(gs, gsl, acc, ticket, tl, tv);
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        spmv_store_row<MODE>(tv[q] && row < n, row, yv[q], y);
    }
    PSK_SPMV_PROF_AT(2);
}

// ---- Pair-row diagonal SpMV (round 6): 16-B accesses, two CONTIGUOUS rows per lane ---------------------
// spmv_diag_kernel gives each lane one row of a slice: every x gather, the y store and the aux loads move 8 B
// per lane, the rate the guide puts at 0.54-0.70x of 16-B accesses (MI355X_MICROARCH.md, L2 table). Here a
// lane owns rows (2l, 2l+1) of a 128-row half-slice, so x[row + d] for both rows is ONE 16-B load (8-B aligned
// when d is odd; the rare pair whose two columns are not adjacent after the shard mapping — it straddles
// column 0, n or the halo — is loaded element-wise), as are y, aux_q and aux_d; the presence bytes are one
// 2-B load. The -1/+1 diagonals: row 2l's +1 and row 2l+1's -1 are the lane's own pair, row 2l's -1 and row
// 2l+1's +1 come from the neighbouring lanes by DPP wave shifts (NB orders only). H half-slices per wave:
//   H = 2: a wave owns a whole 256-row slice = one gridsum tile (4 slices per workgroup): it publishes its
//          tile's slot itself — no LDS combine, no workgroup barrier; the halves' edge columns come from each
//          other by readlane, so one edge load per wave;
//   H = 1: two waves per slice (2 slices per workgroup), the tile's four wave totals combined in LDS as
//          spmv_publish_multi does.
// Bits: y as spmv_diag_kernel (each row summed from 0.0 in stored order). p.Ap: the tile sum of the one-row
// kernels is ((T0 + T1) + T2) + T3 over their wave totals T_w = wave_total over 64 rows; a lane here holds
// the first level of that tree (a_{2l} + a_{2l+1}), and diag_pair_totals runs the remaining levels in the same
// operand pairs, so p.Ap is bit-identical to the CSR, sliced and one-row diagonal kernels.

// 16-B accesses at 8-B alignment (x + row + d with d odd; aux arrays that are column views)
typedef double dv2u __attribute__((ext_vector_type(2), aligned(8)));
__device__ __forceinline__ dv2 ldu2(const double *p) {
    const dv2u v = *reinterpret_cast<const dv2u *>(p);
    return dv2{v.x, v.y};
}
__device__ __forceinline__ dv2 ldu2nt(const double *p) {
    const dv2u v = __builtin_nontemporal_load(reinterpret_cast<const dv2u *>(p));
    return dv2{v.x, v.y};
}
__device__ __forceinline__ void stu2(double *p, dv2 v) { *reinterpret_cast<dv2u *>(p) = dv2u{v.x, v.y}; }
__device__ __forceinline__ void stu2nt(double *p, dv2 v) {
    __builtin_nontemporal_store(dv2u{v.x, v.y}, reinterpret_cast<dv2u *>(p));
}

// the wave totals of the two 64-row halves of a 128-row half-slice whose lane l holds v = a_{2l} + a_{2l+1}:
// wave_total's levels after its first (quad_perm [1,0,3,2] on a_{2l}, a_{2l+1}) in the same operand pairs —
//   quad sums: lanes 2j, 2j+1 of the pair layout hold the one-row layout's quad j;
//   wave_total's row_ror 4 then row_ror 8 leave ((Q0 + Q3) + (Q2 + Q1)) in lane 0 of each 16-lane row: here a
//   row's four quads are lanes 8r..8r+7, so row_half_mirror puts Q0 + Q3 in lane 8r and Q2 + Q1 in lane 8r+4,
//   and row_shl 4 adds the latter to the former;
//   the four row totals of a one-row wave (its lanes 0/16/32/48) are lanes 0/8/16/24 (first half) and
//   32/40/48/56 (second half), added in that order.
__device__ __forceinline__ double lane_f64(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ void diag_pair_totals(double v, double &t0, double &t1) {
    v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f64<0x141>(v);   // row_half_mirror
    v += dpp_f64<0x104>(v);   // row_shl:4
    t0 = ((lane_f64(v, 0) + lane_f64(v, 8)) + lane_f64(v, 16)) + lane_f64(v, 24);
    t1 = ((lane_f64(v, 32) + lane_f64(v, 40)) + lane_f64(v, 48)) + lane_f64(v, 56);
}

// x at the columns of rows r, r + 1 on diagonal offset d (the diag_col mapping): one 16-B load at the pair's
// first column when the two columns are adjacent and in range. The rare pair that is not (it straddles column
// 0 or n, or a shard's halo) is marked in `fix` and re-read element-wise by diag_pair_fix once every load of
// the wave has been issued and waited for: a fix-up branch between the loads put a vmcnt wait (the pair load
// and the element loads share their destination registers) in front of every later gather
struct PairFix {
    int64_t c0, c1;   // the clamped columns (diag_col's clamp)
    bool bad;         // not one 16-B pair
};
__device__ __forceinline__ dv2 diag_pair_x(const DiagDesc &dd, int64_t n, int64_t r, int64_t d,
                                           const double *__restrict__ x, PairFix &f) {
    int64_t c0 = r + d, c1 = c0 + 1;
    c0 += c0 < 0 ? dd.lo : (c0 >= n ? dd.hi : 0);
    c1 += c1 < 0 ? dd.lo : (c1 >= n ? dd.hi : 0);
    f.bad = !(c1 == c0 + 1 && c0 >= 0 && c1 < dd.ncols);
    f.c0 = c0 < 0 ? 0 : (c0 >= dd.ncols ? dd.ncols - 1 : c0);
    f.c1 = c1 < 0 ? 0 : (c1 >= dd.ncols ? dd.ncols - 1 : c1);
    const int64_t a = c0 < 0 ? 0 : (c0 > dd.ncols - 2 ? dd.ncols - 2 : c0);   // ncols >= 2 (host check)
    return ldu2(x + a);
}
__device__ __forceinline__ void diag_pair_fix(dv2 &v, const PairFix &f, const double *__restrict__ x) {
    if (f.bad) {
        v.x = x[f.c0];
        v.y = x[f.c1];
    }
}

// 8 workgroups per CU (<= 64 VGPRs) where that does not spill: the H = 2 forms of the modes with aux loads keep
// more in flight and are left at 4
template <int MODE, int NB, int H>
__global__ __launch_bounds__(kBlock, (H == 2 && MODE != kSpmvPlain && MODE != kSpmvDot) ? 4 : 8) void spmv_diagp_kernel(
    int64_t n, const uint8_t *__restrict__ mask, DiagDesc dd, const double *__restrict__ x, double *__restrict__ y,
    const double *__restrict__ aux_d, const double *__restrict__ aux_q, GridSum gs, const int32_t *__restrict__ done,
    TileMap tm, int64_t ntiles) {
    constexpr int KM = 5;
    static_assert(NB == 1 || NB == 2, "the 5-diagonal DPP orders");
    static_assert(H == 1 || H == 2, "half-slices per wave");
    constexpr int JD = NB == 1 ? 0 : 2, JM1 = NB == 1 ? 3 : 1, JP1 = NB == 1 ? 4 : 3;
    constexpr int GD = NB == 1 ? 0 : 1;   // the d = 0 pair among the three gathered diagonals
    constexpr int TPB = H == 2 ? kWaves : kWaves / 2;   // slices (gridsum tiles) per workgroup
    constexpr bool JX = MODE == kSpmvJacobiDot;           // gathers of (DInv * q)[c]
    constexpr bool EQ = MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot;
    const int32_t dnv = (done ? done : &g_spmv_never_done)[spmv_vzero()];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t grp = tile_of_block(tm);
    const int64_t t = grp * TPB + (H == 2 ? wave : wave >> 1);   // this wave's slice
    const bool tv = t < ntiles;                                   // wave-uniform
    const int64_t tl = tv ? t : ntiles - 1;
    const int64_t r0 = tl * kSlice + (H == 2 ? 0 : 128 * (wave & 1));   // first row of the wave's first half
    uint32_t mk[H];
    dv2 xv[H][3], dg[H][3], eq[H];
    PairFix fx[H][3];
    double xe, de = 1.0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int64_t row = r0 + 128 * h + 2 * lane;
        mk[h] = __builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(mask + row));   // padded slices
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int64_t row = r0 + 128 * h + 2 * lane;
        int g = 0;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (j == JM1 || j == JP1) continue;   // from the d = 0 pair (own lane and neighbours)
            xv[h][g] = diag_pair_x(dd, n, row, dd.d[j], x, fx[h][g]);
            if (JX) dg[h][g] = diag_pair_x(dd, n, row, dd.d[j], aux_d, fx[h][g]);
            ++g;
        }
        eq[h] = dv2{0.0, 0.0};
        if (EQ) eq[h] = ldu2(aux_q + (row + 1 < n ? row : (n >= 2 ? n - 2 : 0)));   // n >= 2 (host check)
    }
    {   // the wave's edge columns: lane 0 x[first row - 1], lane 63 x[last row + 1]; the other lanes re-read
        // their own x[row] (one load instruction, no branch)
        const int64_t er = lane == 0 ? r0 - 1 : (lane == 63 ? r0 + 128 * H : r0 + 2 * lane);
        const int64_t c = diag_col_off(dd, n, er, 0);
        xe = x[c];
        if (JX) de = aux_d[c];
    }
    constexpr bool PUB = MODE != kSpmvPlain && MODE != kSpmvAdd;
    const bool pub = PUB && spmv_publishes<MODE>(gs);
    const bool drawer = H == 2 || (wave & 1) == 0;   // the wave that draws its slice's ticket
    // (drawn after the loads: drawn before them, its return held the loads' consumption back — in-loop SpMV
    // 0.049 -> 0.060 ms at N = 10M, profiles/r6_diagp_epilogue_ab.txt)
    uint32_t ticket = 0;
    if (pub && tv && drawer && gs.grp_log2 >= 0 && lane == 0)
        ticket = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tl, gs.grp_log2)));
    if (__builtin_amdgcn_readfirstlane(dnv) != 0) {   // uniform: the solve has stopped; tickets handed back
#pragma unroll
        for (int h = 0; h < H; ++h) {
            __asm__ volatile("" ::"v"(mk[h]));
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                __asm__ volatile("" ::"v"(xv[h][g].x), "v"(xv[h][g].y));
                if (JX) __asm__ volatile("" ::"v"(dg[h][g].x), "v"(dg[h][g].y));
            }
            if (EQ) __asm__ volatile("" ::"v"(eq[h].x), "v"(eq[h].y));
        }
        __asm__ volatile("" ::"v"(xe), "v"(de));
        if (pub && tv && drawer && gs.grp_log2 >= 0 && lane == 0)
            __hip_atomic_fetch_sub(gridsum_counter(gs, gridsum_group_of(tl, gs.grp_log2)), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __shared__ GridSumTile<1> gsl[H == 1 ? TPB : 1];
    if (H == 1 && pub) {
        if (threadIdx.x < TPB) gsl[threadIdx.x].cnt = 0;
        __syncthreads();
    }
    if (pub && threadIdx.x == 0 && blockIdx.x == 0 && (gs.nt + TPB - 1) / TPB != gridDim.x) atomicOr(gs.err, 2);
    // the rare pairs that are not one 16-B load, then (DInv*q)[c] products (JX), all after every load was issued
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            diag_pair_fix(xv[h][g], fx[h][g], x);
            if (JX) {
                diag_pair_fix(dg[h][g], fx[h][g], aux_d);
                xv[h][g].x = dg[h][g].x * xv[h][g].x;   // (DInv*q)[c], rounded
                xv[h][g].y = dg[h][g].y * xv[h][g].y;
            }
        }
    if (JX) xe = de * xe;
    // the +-1 neighbours: g = GD is the d = 0 pair (x[row], x[row + 1]) of every lane
    double xl[H], xr[H];   // x[row - 1] of the lane's first row, x[row + 2] of its second
    if constexpr (H == 2) {
        const double a63 = lane_f64(xv[0][GD].y, 63), b0 = lane_f64(xv[1][GD].x, 0);
        xl[0] = wave_shift1<true>(xv[0][GD].y, xe);                    // lane 0: the loaded x[r0 - 1]
        xr[0] = wave_shift1<false>(xv[0][GD].x, b0);                   // lane 63: row 128 = half 1's lane 0
        xl[1] = wave_shift1<true>(xv[1][GD].y, a63);                   // lane 0: row 127 = half 0's lane 63
        xr[1] = wave_shift1<false>(xv[1][GD].x, xe);                   // lane 63: the loaded x[r0 + 256]
    } else {
        xl[0] = wave_shift1<true>(xv[0][GD].y, xe);
        xr[0] = wave_shift1<false>(xv[0][GD].x, xe);
    }
    double acc[H];
    dv2 yv[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int64_t row = r0 + 128 * h + 2 * lane;
        // the five diagonals' x of each row in j order (stored order)
        double c0[KM], c1[KM];
        int g = 0;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (j == JM1) {
                c0[j] = xl[h];
                c1[j] = xv[h][GD].x;
            } else if (j == JP1) {
                c0[j] = xv[h][GD].y;
                c1[j] = xr[h];
            } else {
                c0[j] = xv[h][g].x;
                c1[j] = xv[h][g].y;
                ++g;
            }
        }
        const uint32_t m0 = mk[h] & 0xffu, m1 = mk[h] >> 8;
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int j = 0; j < KM; ++j) {   // stored order, rounded product; absent diagonals by a select
            const double u0 = s0 + dd.v[j] * c0[j], u1 = s1 + dd.v[j] * c1[j];
            s0 = ((m0 >> j) & 1u) ? u0 : s0;
            s1 = ((m1 >> j) & 1u) ? u1 : s1;
        }
        const bool has0 = tv && row < n, has1 = tv && row + 1 < n;
        double e0 = eq[h].x, e1 = eq[h].y;
        if (EQ && row + 1 >= n) {   // the last pair of an odd n: aux_q was loaded one row early
            e0 = eq[h].y;
            e1 = 0.0;
        }
        if (MODE == kSpmvDot) {   // x[row]: the d = 0 gather when the row stores its diagonal
            const bool f0 = (m0 >> JD) & 1u, f1 = (m1 >> JD) & 1u;
            e0 = f0 ? c0[JD] : 0.0;
            e1 = f1 ? c1[JD] : 0.0;
            if (!f0 && has0) e0 = x[row];   // rare: a row without its diagonal
            if (!f1 && has1) e1 = x[row + 1];
        }
        double a0, a1;
        yv[h].x = spmv_row_value<MODE>(has0, s0, e0, a0);
        yv[h].y = spmv_row_value<MODE>(has1, s1, e1, a1);
        acc[h] = a0 + a1;   // wave_total's first level
    }
    if (pub && tv) {
        double w[2 * H];
#pragma unroll
        for (int h = 0; h < H; ++h) diag_pair_totals(acc[h], w[2 * h], w[2 * h + 1]);
        bool reduce = false;
        uint32_t tk = 0;
        double s = 0.0;
        if (H == 2) {   // the wave is the tile
            s = ((w[0] + w[1]) + w[2]) + w[3];
            tk = __builtin_amdgcn_readfirstlane(ticket);
            reduce = true;
        } else {        // two waves per tile: the later one publishes
            GridSumTile<1> &L = gsl[wave >> 1];
            const int hb = wave & 1;
            uint32_t old = 0;
            if (lane == 0) {
                L.part[2 * hb] = w[0];
                L.part[2 * hb + 1] = w[1];
                if (hb == 0) L.ticket = ticket;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                old = atomicAdd(&L.cnt, 1u);
            }
            if (__builtin_amdgcn_readfirstlane(old) == 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                s = ((L.part[0] + L.part[1]) + L.part[2]) + L.part[3];
                tk = L.ticket;
                reduce = true;
            }
        }
        if (reduce) {
            if (gs.grp_log2 < 0) {
                if (lane == 0) gridsum_put(gs.gslots + tl, s);
                gridsum_final_wave<1>(gs);
            } else {
                if (lane == 0) gridsum_put(gs.slots + gridsum_slot(gs, tl), s);
                const int64_t g = gridsum_group_of(tl, gs.grp_log2);
                int64_t base;
                const int64_t cnt = gridsum_members(gs, g, base);
                if (tk == (uint32_t)(cnt - 1)) {
                    double r[1];
                    gridsum_take<1, 64>(gs.slots, g << gs.grp_log2, cnt, gs.err, nullptr, r);
                    if (lane == 0) {
                        gridsum_reset(gridsum_counter(gs, g));
                        gridsum_put(gs.gslots + g, r[0]);
                    }
                    gridsum_final_wave<1>(gs);
                }
            }
        }
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {   // y after the dot epilogue (spmv_row_value)
        const int64_t row = r0 + 128 * h + 2 * lane;
        if (!tv || row >= n) continue;
        if (row + 1 < n) {
            if (MODE == kSpmvResid || MODE == kSpmvAdd) stu2(y + row, yv[h]);
            else stu2nt(y + row, yv[h]);
        } else {
            spmv_store_row<MODE>(true, row, yv[h].x, y);
        }
    }
}

// ---- the PCG init fused into the first SpMV (round 5; diagonal layout in a DPP order, unsharded, Jacobi with one
// DInv value or none): p_0 = M b (PCGSolver.py:98) computed where this SpMV gathers it (xs * b[c]: xs = the DInv
// value, or 1.0), Ap_0 = A p_0 (:111) and the three sums [p_0.Ap_0, b.b, u.r] (:113, :86, :102) through the
// SpMV's tile epilogue; the wave that finishes them runs the init's state logic (PcgInitFin, sums 1 and 2), and
// p_0 is stored for K3. One launch instead of pcg_init_kernel + the SpMV of iteration 0 (b read once, not b and
// then p_0). b.b and u.r have pcg_init_kernel's bits (same 256-row tiles, same per-row products, wave totals in
// wave order), p_0.Ap_0 and Ap_0 the SpMV's (p_0 = xs * b is the product pcg_init_kernel stores).
template <int NB>
__global__ __launch_bounds__(kBlock) void pcg_init_diag_kernel(int64_t n, const uint8_t *__restrict__ mask, DiagDesc dd,
                                                               const double *__restrict__ b, double xs,
                                                               double *__restrict__ p, double *__restrict__ y,
                                                               GridSum gs, PcgInitFin fin, TileMap tm, int64_t ntiles) {
    constexpr int TPW = kDiagTpw, KM = 5;
    static_assert(NB == 1 || NB == 2, "the DPP orders of spmv_diag_kernel");
    constexpr int JD = NB == 1 ? 0 : 2, JM1 = NB == 1 ? 3 : 1, JP1 = NB == 1 ? 4 : 3;
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t grp = tile_of_block(tm);
    int64_t tl[TPW];
    bool tv[TPW];
    uint32_t mk[TPW];
    double xv[TPW][KM], xe[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t t = grp * TPW + q;
        tv[q] = t < ntiles;
        tl[q] = tv[q] ? t : ntiles - 1;
        mk[q] = __builtin_nontemporal_load(mask + tl[q] * kSlice + tid);
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            if (j == JM1 || j == JP1) continue;
            xv[q][j] = b[diag_col(dd, n, row, j)];
        }
        xe[q] = b[diag_col_off(dd, n, row, lane == 0 ? -1 : (lane == 63 ? 1 : 0))];
    }
    uint32_t ticket[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        ticket[q] = 0;
        if (tv[q] && gs.grp_log2 >= 0 && tid == 0)
            ticket[q] = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tl[q], gs.grp_log2)));
    }
    __shared__ GridSumTile<3> gsl[TPW];
    if (tid < TPW) gsl[tid].cnt = 0;
    if (tid == 0 && blockIdx.x == 0 && (gs.nt + TPW - 1) / TPW != gridDim.x) atomicOr(gs.err, 2);
    __syncthreads();
    double acc[TPW][3], yv[TPW], pv[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        const bool has = tv[q] && row < n;
        const double braw = xv[q][JD];   // b[row] (the d = 0 column of a row < n is the row itself)
#pragma unroll
        for (int j = 0; j < KM; ++j)
            if (j != JM1 && j != JP1) xv[q][j] = xs * xv[q][j];   // u = precond.applyRight(r)  :98
        xe[q] = xs * xe[q];
        xv[q][JM1] = wave_shift1<true>(xv[q][JD], xe[q]);
        xv[q][JP1] = wave_shift1<false>(xv[q][JD], xe[q]);
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < KM; ++j) {   // stored order, rounded product (spmv_diag_kernel)
            const double t = sum + dd.v[j] * xv[q][j];
            sum = ((mk[q] >> j) & 1u) ? t : sum;
        }
        pv[q] = xv[q][JD];
        yv[q] = sum;
        acc[q][0] = has ? pv[q] * sum : 0.0;    // np.dot(p, Ap)  :113 (spmv_row_value's eq * sum)
        acc[q][1] = has ? braw * braw : 0.0;    // self.norm(b)   :86
        acc[q][2] = has ? pv[q] * braw : 0.0;   // np.dot(u, r)   :102
    }
    gridsum_tiles_publish<TPW, 3>(gs, gsl, acc, ticket, tl, tv, fin);
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t row = tl[q] * kSlice + tid;
        if (tv[q] && row < n) {
            __builtin_nontemporal_store(yv[q], y + row);
            p[row] = pv[q];
        }
    }
}

// (Round 5 also built K3 fused into the next SpMV — pcg_fused_kernel, 33 B/row in one launch instead of 24 + 17 in
// two, bit-identical — and a persistent form of spmv_diag_kernel; both measured no faster (profiles/
// r5_pcg_fused_ab.txt, r5_diag_tpw_ab.txt) and were removed from the product library in round 6.)


// Diagonal-layout detection: row `row`'s stored entries must be, in order, entries of strictly increasing
// diagonals j with column diag_col's mapping and value v_j; the presence byte is written (0 past n) and
// any violation sets *bad.
__global__ __launch_bounds__(kBlock) void diag_detect_kernel(int64_t n, const int32_t *__restrict__ rowptr,
                                                             const int32_t *__restrict__ colidx,
                                                             const double *__restrict__ vals, DiagDesc dd,
                                                             uint8_t *__restrict__ mask, int64_t npad,
                                                             int32_t *__restrict__ bad) {
    const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (row >= npad) return;
    uint32_t mk = 0;
    if (row < n) {
        int j = 0;
        bool ok = true;
        for (int32_t e = rowptr[row]; e < rowptr[row + 1] && ok; ++e) {
            const int64_t c = colidx[e];
            const double v = vals[e];
            while (j < dd.K) {
                int64_t cj = row + dd.d[j];
                cj += cj < 0 ? dd.lo : (cj >= n ? dd.hi : 0);
                if (cj == c && same_bits(v, dd.v[j])) break;
                ++j;
            }
            if (j == dd.K) ok = false;
            else mk |= 1u << j++;
        }
        if (!ok) atomicOr(bad, 1);
    }
    mask[row] = (uint8_t)mk;
}

// General sliced layout (per-slice widths, offsets and formats loaded from the slice header).
// DK: dictionary size class (0 = double values, 2 / 4 / 8 entries).
template <int MODE, int DK>
__global__ __launch_bounds__(kBlock) void spmv_sliced_kernel(
    int64_t n, const int64_t *__restrict__ soff, const int64_t *__restrict__ swoff, const int8_t *__restrict__ sfmt,
    const int32_t *__restrict__ scol, const int32_t *__restrict__ spcol, const double *__restrict__ sval,
    const double *__restrict__ sdict,
    const double *__restrict__ x, double *__restrict__ y, const double *__restrict__ aux_d,
    const double *__restrict__ aux_q, GridSum gs, const int32_t *__restrict__ done, TileMap tm) {
    if (done != nullptr && *done != 0) return;
    const int tid = threadIdx.x;
    const int64_t t = tile_of_block(tm), row = t * kSlice + tid;
    const bool has = row < n;
    const int64_t o = soff[t];
    const int w = (int)((soff[t + 1] - o) / kSlice);
    const bool packed = sfmt[t] != 0;   // uniform across the workgroup
    const int64_t wo = swoff[t];
    const int32_t *pword = spcol + wo;                                         // packed column words
    const int32_t *vword = pword + (packed ? (int64_t)((w + 1) / 2) * kSlice : 0);   // dictionary indices
    const DictRegs dv = load_dict<DK>(sdict);
    __shared__ GridSumTile<1> gsl;
    const uint32_t ticket = spmv_begin<MODE>(gs, gsl, t);
    const int32_t row32 = (int32_t)row;
    double eq = 0.0;
    if (has) {
        if (MODE == kSpmvDot && w > kSliceRegs) eq = x[row];   // register path: diag_x below
        if (MODE == kSpmvResid || MODE == kSpmvAdd || MODE == kSpmvJacobiDot || MODE == kSpmvPlainDot)
            eq = aux_q[row];
    }
    double sum = 0.0;
    if (w <= kSliceRegs) {
        int32_t cc[kSliceRegs];
        double vv[kSliceRegs], xv[kSliceRegs];
#pragma unroll
        for (int j = 0; j < kSliceRegs; ++j) {
            cc[j] = -1;
            vv[j] = 0.0;
        }
        // the slice's whole stream first (w and packed are uniform): values by pairs (or dictionary
        // index words), then columns
        int32_t vw[kSliceRegs / 4];
        if (DK > 0) {
#pragma unroll
            for (int q = 0; q < kSliceRegs / 4; ++q) vw[q] = 4 * q < w ? ld_stream(vword + q * kSlice + tid) : 0;
        } else {
#pragma unroll
            for (int p = 0; p < kSliceRegs / 2; ++p) {
                if (2 * p + 1 < w) {
                    const dv2 v2 =
                        __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(sval + o + 2 * p * kSlice) + tid);
                    vv[2 * p] = v2.x;
                    vv[2 * p + 1] = v2.y;
                } else if (2 * p < w) {
                    vv[2 * p] = ld_stream(sval + o + 2 * p * kSlice + tid);
                }
            }
        }
        if (packed) {
#pragma unroll
            for (int p = 0; p < kSliceRegs / 2; ++p)
                if (2 * p < w) {
                    const int32_t word = ld_stream(pword + p * kSlice + tid);
                    cc[2 * p] = unpack_delta(row32, (int16_t)(word & 0xffff));
                    cc[2 * p + 1] = unpack_delta(row32, (int16_t)(word >> 16));
                }
        } else {
#pragma unroll
            for (int j = 0; j < kSliceRegs; ++j)
                if (j < w) cc[j] = ld_stream(scol + o + j * kSlice + tid);
        }
        if (DK > 0) {
#pragma unroll
            for (int j = 0; j < kSliceRegs; ++j)
                if (j < w) vv[j] = dict_pick<DK>(dv, ((uint32_t)vw[j >> 2] >> (8 * (j & 3))) & 0xff);
        }
#pragma unroll
        for (int j = 0; j < kSliceRegs; ++j) {   // then every gather
            xv[j] = 0.0;
            if (cc[j] >= 0) {
                xv[j] = x[cc[j]];
                if (MODE == kSpmvJacobiDot) xv[j] = aux_d[cc[j]] * xv[j];   // (DInv*q)[c], rounded
            }
        }
#pragma unroll
        for (int j = 0; j < kSliceRegs; ++j)
            if (cc[j] >= 0) sum = sum + vv[j] * xv[j];   // stored order, rounded product
        if (MODE == kSpmvDot) eq = diag_x<kSliceRegs>(cc, xv, row32, x, has);
    } else {
        for (int j = 0; j < w; ++j) {
            int32_t c;
            if (packed) {
                const int32_t word = ld_stream(pword + (int64_t)(j >> 1) * kSlice + tid);
                c = unpack_delta(row32, (int16_t)((j & 1) ? (word >> 16) : (word & 0xffff)));
            } else {
                c = ld_stream(scol + o + (int64_t)j * kSlice + tid);
            }
            if (c < 0) break;   // only padding follows a row's last entry
            double xx = x[c];
            if (MODE == kSpmvJacobiDot) xx = aux_d[c] * xx;
            const double v =
                DK > 0 ? dict_pick<DK>(dv, ((uint32_t)ld_stream(vword + (int64_t)(j >> 2) * kSlice + tid) >> (8 * (j & 3))) &
                                               0xff)
                       : ld_stream(sval + sliced_vpos(o, j, w, tid));
            sum = sum + v * xx;
        }
    }
    double acc;
    const double yv = spmv_row_value<MODE>(has, sum, eq, acc);
    if (spmv_publishes<MODE>(gs)) spmv_publish(gs, gsl, acc, ticket, t);
    spmv_store_row<MODE>(has, row, yv, y);
}

// per slice: widest row, and the largest |column - row| of its entries (saturated to int32)
__global__ __launch_bounds__(kBlock) void sliced_shape_kernel(int64_t n, const int32_t *__restrict__ rowptr,
                                                              const int32_t *__restrict__ colidx,
                                                              int32_t *__restrict__ width, int32_t *__restrict__ span) {
    __shared__ int32_t sh[2 * kWaves];
    const int64_t row = (int64_t)blockIdx.x * kSlice + threadIdx.x;
    int32_t len = 0, dmax = 0;
    if (row < n) {
        const int32_t a = rowptr[row], b = rowptr[row + 1];
        len = b - a;
        for (int32_t e = a; e < b; ++e) {
            int64_t d = (int64_t)colidx[e] - row;
            d = d < 0 ? -d : d;
            const int32_t ds = d > INT32_MAX ? INT32_MAX : (int32_t)d;
            dmax = ds > dmax ? ds : dmax;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t v = __shfl_xor(len, o, 64), u = __shfl_xor(dmax, o, 64);
        len = v > len ? v : len;
        dmax = u > dmax ? u : dmax;
    }
    if ((threadIdx.x & 63) == 0) {
        sh[threadIdx.x >> 6] = len;
        sh[kWaves + (threadIdx.x >> 6)] = dmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t m = sh[0], dm = sh[kWaves];
        for (int i = 1; i < kWaves; ++i) {
            m = sh[i] > m ? sh[i] : m;
            dm = sh[kWaves + i] > dm ? sh[kWaves + i] : dm;
        }
        width[blockIdx.x] = m;
        span[blockIdx.x] = dm;
    }
}

// One detection pass for the value dictionary: every wave that meets a value (bit pattern) not in
// dict[0, nd) offers its first such value; the first kDictCand offers land in cand. No offers =
// the dictionary is complete.
__global__ __launch_bounds__(kBlock) void dict_scan_kernel(int64_t nnz, const double *__restrict__ vals,
                                                           const double *__restrict__ dict, int nd,
                                                           int32_t *__restrict__ ncand, double *__restrict__ cand) {
    __shared__ double dl[kDictMax];
    if (threadIdx.x < nd) dl[threadIdx.x] = dict[threadIdx.x];
    __syncthreads();
    double mine = 0.0;
    bool has = false;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * kBlock) {
        const double v = vals[i];
        bool found = false;
        for (int k = 0; k < nd && !found; ++k) found = same_bits(v, dl[k]);
        if (!found) {
            mine = v;
            has = true;
            break;
        }
    }
    const uint64_t m = __ballot(has);
    if (m != 0 && (threadIdx.x & 63) == __builtin_ctzll(m)) {
        const int32_t slot = atomicAdd(ncand, 1);
        if (slot < kDictCand) cand[slot] = mine;
    }
}

// one workgroup per slice, one lane per row (lanes past n write padding): coalesced stores
__global__ __launch_bounds__(kBlock) void sliced_fill_kernel(int64_t n, const int32_t *__restrict__ rowptr,
                                                             const int32_t *__restrict__ colidx,
                                                             const double *__restrict__ vals,
                                                             const int64_t *__restrict__ soff,
                                                             const int64_t *__restrict__ swoff,
                                                             const int8_t *__restrict__ sfmt, int32_t *__restrict__ scol,
                                                             int32_t *__restrict__ spcol, double *__restrict__ sval,
                                                             const double *__restrict__ sdict, int nd,
                                                             int compact) {
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x, row = t * kSlice + tid;
    const int64_t o = soff[t];
    const int w = (int)((soff[t + 1] - o) / kSlice);
    const bool packed = sfmt[t] != 0;
    const int64_t a = row < n ? rowptr[row] : 0;
    const int64_t len = row < n ? rowptr[row + 1] - a : 0;
    for (int j = 0; j < w; ++j) {
        if (!sdict) sval[sliced_vpos(o, j, w, tid)] = j < len ? vals[a + j] : 0.0;
        if (!packed) scol[o + (int64_t)j * kSlice + tid] = j < len ? colidx[a + j] : -1;
    }
    if (sdict && !compact) {   // index words; padding slots index entry 0 (never read: their column is padding)
        int32_t *vword = spcol + swoff[t] + (packed ? (int64_t)((w + 1) / 2) * kSlice : 0);
        for (int q = 0; 4 * q < w; ++q) {
            uint32_t word = 0;
            for (int b = 0; b < 4; ++b) {
                const int j = 4 * q + b;
                uint32_t k = 0;
                if (j < len)
                    while (k + 1 < (uint32_t)nd && !same_bits(sdict[k], vals[a + j])) ++k;
                word |= k << (8 * b);
            }
            vword[(int64_t)q * kSlice + tid] = (int32_t)word;
        }
    }
    if (packed)
        for (int p = 0; 2 * p < w; ++p) {
            const int j0 = 2 * p, j1 = 2 * p + 1;
            const int16_t d0 = j0 < len ? (int16_t)(colidx[a + j0] - row) : kPad16;
            const int16_t d1 = j1 < len ? (int16_t)(colidx[a + j1] - row) : kPad16;
            uint32_t hi = (uint16_t)d1;
            if (compact && j1 == w) {   // the free half: bit j = entry j's dictionary index (nd <= 2)
                hi = 0;
                for (int j = 0; j < w && j < len; ++j)
                    if (nd > 1 && !same_bits(sdict[0], vals[a + j])) hi |= 1u << j;   // the index word's k
            }
            spcol[swoff[t] + (int64_t)p * kSlice + tid] = (int32_t)((uint32_t)(uint16_t)d0 | (hi << 16));
        }
}

void sliced_free(psk_csr *A) {
    void *ptrs[] = {A->sl_off, A->sl_woff, A->sl_fmt, A->sl_col, A->sl_pcol, A->sl_val, A->sl_dict};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    A->sl_off = nullptr;
    A->sl_woff = nullptr;
    A->sl_fmt = nullptr;
    A->sl_col = nullptr;
    A->sl_pcol = nullptr;
    A->sl_val = nullptr;
    A->sl_dict = nullptr;
    A->sl_dict_n = 0;
    A->sl_uniform_w = 0;
    A->sl_compact = 0;
    A->sl_slots = 0;
    A->sl_packed_slots = 0;
    A->sl_stream_bytes = 0;
}

void diag_free(psk_csr *A) {
    if (A->dg_mask) (void)hipFree(A->dg_mask);
    A->dg_mask = nullptr;
    A->dg_K = 0;
    A->dg_jd = -1;
}

static DiagDesc diag_desc(const psk_csr *A) {
    DiagDesc dd{};
    for (int j = 0; j < kDiagMax; ++j) {
        dd.d[j] = A->dg_d[j];
        dd.v[j] = A->dg_v[j];
    }
    dd.lo = A->dg_lo;
    dd.hi = A->dg_hi;
    dd.ncols = A->ncols;
    dd.K = A->dg_K;
    dd.jd = A->dg_jd;
    return dd;
}

// The diagonal layout of A when it has one (see spmv_diag_kernel): the diagonals and their values are
// read off one full-width row of owned columns, the halo mapping of a shard from its column count, and then
// EVERY row is checked against them on the device. Quietly leaves A alone when the rule does not hold
// (force: fails with PSK_ERR_UNSUPPORTED).
static int diag_build(psk_csr *A, hipStream_t s, bool force) {
    auto no = [&](const char *why) { return force ? fail(PSK_ERR_UNSUPPORTED, std::string("diagonal layout: ") + why) : PSK_OK; };
    const int64_t n = A->n, nt = (n + kSlice - 1) / kSlice;
    if (n == 0 || A->nnz == 0) return no("empty matrix");
    if (nt > INT32_MAX) return no("too many slices");
    DevBuf tmp;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{tmp};
    PSK_TRY(tmp.ensure((size_t)nt * 2 * sizeof(int32_t) + 64));
    int32_t *dw = tmp.as<int32_t>(), *dspan = dw + nt;
    int32_t *dbad = dw + 2 * nt;
    hipLaunchKernelGGL(sliced_shape_kernel, dim3((unsigned)nt), dim3(kBlock), 0, s, n, A->rowptr, A->colidx, dw, dspan);
    PSK_HIP(hipGetLastError());
    std::vector<int32_t> wd((size_t)nt);
    PSK_HIP(hipMemcpyAsync(wd.data(), dw, (size_t)nt * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    const int32_t K = *std::max_element(wd.begin(), wd.end());
    if (K < 1 || K > kDiagMax) return no("rows wider than 8 entries");
    // the template row: a row of K entries, all in owned columns, from slices taken from the middle out
    // (a shard's first and last lines reach into its halo)
    std::vector<int32_t> rp(kSlice + 1), cols(K);
    std::vector<double> vals(K);
    int64_t trow = -1;
    for (int64_t tries = 0, i = 0; i < nt && tries < 64 && trow < 0; ++i) {
        const int64_t t = (nt / 2 + i) % nt;
        if (wd[(size_t)t] != K) continue;
        ++tries;
        const int64_t r0 = t * kSlice, nr = std::min<int64_t>(kSlice, n - r0);
        PSK_HIP(hipMemcpy(rp.data(), A->rowptr + r0, (size_t)(nr + 1) * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < nr && trow < 0; ++r) {
            if (rp[(size_t)r + 1] - rp[(size_t)r] != K) continue;
            PSK_HIP(hipMemcpy(cols.data(), A->colidx + rp[(size_t)r], (size_t)K * 4, hipMemcpyDeviceToHost));
            bool owned = true;
            for (int j = 0; j < K; ++j) owned = owned && cols[(size_t)j] >= 0 && cols[(size_t)j] < n;
            if (!owned) continue;
            PSK_HIP(hipMemcpy(vals.data(), A->vals + rp[(size_t)r], (size_t)K * 8, hipMemcpyDeviceToHost));
            trow = r0 + r;
        }
    }
    if (trow < 0) return no("no full-width row of owned columns");
    DiagDesc dd{};
    dd.K = K;
    dd.jd = -1;
    int64_t dmin = 0;
    for (int j = 0; j < K; ++j) {
        const int64_t d = (int64_t)cols[(size_t)j] - trow;
        for (int i = 0; i < j; ++i)
            if (dd.d[i] == d) return no("repeated column in a row");
        dd.d[j] = (int32_t)d;
        dd.v[j] = vals[(size_t)j];
        if (d == 0) dd.jd = j;
        dmin = std::min(dmin, d);
    }
    // halo mapping of a row-block shard with columns [owned | below | above] (psk_csr_create_fd2d_dist):
    // the lines below hold -dmin columns; a shard with one halo has it right after the owned block
    const int64_t halo = A->ncols - n;
    dd.lo = halo > 0 ? n - dmin : 0;
    dd.hi = halo > 0 && halo == -2 * dmin ? -dmin : 0;
    dd.ncols = A->ncols;
    uint8_t *mask = nullptr;
    if (hipMalloc(&mask, (size_t)nt * kSlice) != hipSuccess) {
        (void)hipGetLastError();
        return force ? fail(PSK_ERR_ALLOC, "diagonal layout: hipMalloc") : PSK_OK;
    }
    PSK_HIP(hipMemsetAsync(dbad, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(diag_detect_kernel, dim3((unsigned)nt), dim3(kBlock), 0, s, n, A->rowptr, A->colidx, A->vals, dd,
                       mask, nt * kSlice, dbad);
    int32_t bad = 0;
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, dbad, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess || bad) {
        (void)hipFree(mask);
        if (e != hipSuccess) return fail(PSK_ERR_HIP, std::string("diagonal layout: ") + hipGetErrorString(e));
        return no("an entry off the diagonals or with another value");
    }
    sliced_free(A);
    diag_free(A);
    A->dg_mask = mask;
    A->dg_K = K;
    A->dg_jd = dd.jd;
    for (int j = 0; j < kDiagMax; ++j) {
        A->dg_d[j] = j < K ? dd.d[j] : 0;
        A->dg_v[j] = j < K ? dd.v[j] : 0.0;
    }
    A->dg_lo = dd.lo;
    A->dg_hi = dd.hi;
    return PSK_OK;
}

// The distinct values of A (bit patterns) when there are at most kDictMax of them, else empty:
// detection passes over A->vals, each adding every new value it was offered (<= kDictMax + 1 passes,
// one for a matrix of arbitrary values).
static int find_value_dict(const psk_csr *A, hipStream_t s, std::vector<double> &dict) {
    dict.clear();
    if (A->nnz == 0) return PSK_OK;
    DevBuf tmp;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{tmp};
    PSK_TRY(tmp.ensure((size_t)(kDictMax + kDictCand + 1) * sizeof(double)));
    double *ddict = tmp.as<double>(), *dcand = ddict + kDictMax;
    int32_t *dn = reinterpret_cast<int32_t *>(dcand + kDictCand);
    const int64_t blocks = std::min<int64_t>((A->nnz + kBlock - 1) / kBlock, 2048);
    std::vector<double> cand(kDictCand);
    for (int pass = 0; pass <= kDictMax; ++pass) {
        if (!dict.empty())
            PSK_HIP(hipMemcpyAsync(ddict, dict.data(), dict.size() * sizeof(double), hipMemcpyHostToDevice, s));
        PSK_HIP(hipMemsetAsync(dn, 0, sizeof(int32_t), s));
        hipLaunchKernelGGL(dict_scan_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, A->nnz, A->vals, ddict,
                           (int)dict.size(), dn, dcand);
        PSK_HIP(hipGetLastError());
        int32_t nc = 0;
        PSK_HIP(hipMemcpyAsync(&nc, dn, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        PSK_HIP(hipMemcpyAsync(cand.data(), dcand, kDictCand * sizeof(double), hipMemcpyDeviceToHost, s));
        PSK_HIP(hipStreamSynchronize(s));
        if (nc == 0) return PSK_OK;   // every value is in the dictionary
        for (int i = 0; i < std::min(nc, kDictCand); ++i) {
            bool seen = false;
            for (double d : dict) seen = seen || std::memcmp(&d, &cand[(size_t)i], sizeof(double)) == 0;
            if (!seen) dict.push_back(cand[(size_t)i]);
            if ((int)dict.size() > kDictMax) {
                dict.clear();
                return PSK_OK;
            }
        }
    }
    dict.clear();
    return PSK_OK;
}

// Builds the sliced copy of A (pack = allow int16 column deltas, use_dict = index values through a
// dictionary when A has at most kDictMax distinct values; force_dict fails when it has more).
// Unless `force`, only when its stream is no larger than the CSR stream (12 B per entry + 4 B per
// row), i.e. padding costs nothing, and quietly keeps CSR if HBM cannot hold the copy.
static int sliced_build(psk_csr *A, hipStream_t s, bool force, bool pack, bool use_dict, bool force_dict) {
    sliced_free(A);
    diag_free(A);
    std::vector<double> dict;
    if (use_dict) PSK_TRY(find_value_dict(A, s, dict));
    if (force_dict && dict.empty())
        return fail(PSK_ERR_UNSUPPORTED, "sliced layout: more than 8 distinct values, no value dictionary");
    const int64_t nt = (A->n + kSlice - 1) / kSlice;
    if (nt == 0) return PSK_OK;   // nothing to multiply (launch_spmv returns early)
    if (nt > INT32_MAX) return force ? fail(PSK_ERR_UNSUPPORTED, "sliced layout: too many slices") : PSK_OK;
    DevBuf tmp;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{tmp};
    PSK_TRY(tmp.ensure((size_t)nt * 2 * sizeof(int32_t)));
    int32_t *dw = tmp.as<int32_t>(), *dspan = dw + nt;
    hipLaunchKernelGGL(sliced_shape_kernel, dim3((unsigned)nt), dim3(kBlock), 0, s, A->n, A->rowptr, A->colidx, dw,
                       dspan);
    PSK_HIP(hipGetLastError());
    std::vector<int32_t> wd((size_t)nt * 2);
    PSK_HIP(hipMemcpyAsync(wd.data(), tmp.p, (size_t)nt * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    // uniform: every slice padded to the widest when all pack and that pads at most 1% more slots
    // (FD: only the first and last grid lines are narrower) — the kernel then computes every
    // offset from the slice index (PSK_SPMV_UNIFORM=0 disables)
    int64_t wmax = 0, wsum = 0;
    bool all_pack = pack;
    for (int64_t t = 0; t < nt; ++t) {
        wmax = std::max<int64_t>(wmax, wd[(size_t)t]);
        wsum += wd[(size_t)t];
        all_pack = all_pack && wd[(size_t)(nt + t)] <= kMaxDelta16;
    }
    const bool uniform = all_pack && wmax > 0 && wmax <= kSliceRegs && wmax * nt * 100 <= wsum * 101;
    if (uniform)
        for (int64_t t = 0; t < nt; ++t) wd[(size_t)t] = (int32_t)wmax;
    // compact stream: uniform, odd width, a 1-bit value index
    const bool compact = uniform && !dict.empty() && dict.size() <= 2 && (wmax & 1) && wmax <= 15;
    std::vector<int64_t> off((size_t)nt + 1), woff((size_t)nt + 1);
    std::vector<int8_t> fmt((size_t)nt);
    off[0] = 0;
    woff[0] = 0;
    int64_t packed_slots = 0, col_bytes = 0, val_bytes = 0;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t w = wd[(size_t)t];
        off[(size_t)t + 1] = off[(size_t)t] + w * kSlice;
        fmt[(size_t)t] = (pack && wd[(size_t)(nt + t)] <= kMaxDelta16) ? 1 : 0;
        if (fmt[(size_t)t]) packed_slots += w * kSlice;
        col_bytes += (fmt[(size_t)t] ? 4 * ((w + 1) / 2) : 4 * w) * kSlice;
        val_bytes += (dict.empty() ? 8 * w : compact ? 0 : 4 * ((w + 3) / 4)) * kSlice;
        // the word stream: packed column words, then dictionary index words
        const int64_t words = (fmt[(size_t)t] ? (w + 1) / 2 : 0) + (dict.empty() || compact ? 0 : (w + 3) / 4);
        woff[(size_t)t + 1] = woff[(size_t)t] + words * kSlice;
    }
    const int64_t slots = off[(size_t)nt], nwords = woff[(size_t)nt];
    const int64_t wide_slots = slots - packed_slots;
    // matrix bytes one SpMV streams: values (or value indices + dictionary), columns, slice offsets
    // (two arrays) and formats
    const int64_t stream = val_bytes + 8 * (int64_t)dict.size() + col_bytes + (uniform ? 0 : 17 * nt + 16);
    if (!force && stream > 12 * A->nnz + 4 * (A->n + 1)) return PSK_OK;
    const size_t ms = slots > 0 ? (size_t)slots : 1;
    bool ok = hipMalloc(&A->sl_off, (size_t)(nt + 1) * 8) == hipSuccess &&
              hipMalloc(&A->sl_woff, (size_t)(nt + 1) * 8) == hipSuccess &&
              hipMalloc(&A->sl_fmt, (size_t)nt) == hipSuccess;
    if (ok && dict.empty()) ok = hipMalloc(&A->sl_val, ms * 8) == hipSuccess;              // indexed by slot
    if (ok && wide_slots > 0) ok = hipMalloc(&A->sl_col, ms * 4) == hipSuccess;            // indexed by slot
    if (ok && nwords > 0) ok = hipMalloc(&A->sl_pcol, (size_t)nwords * 4) == hipSuccess;   // from sl_woff[t]
    if (ok && !dict.empty()) ok = hipMalloc(&A->sl_dict, kDictMax * 8) == hipSuccess;   // padded: the kernel
                                                                                         // reads its size class
    if (!ok) {
        (void)hipGetLastError();
        sliced_free(A);
        return force ? fail(PSK_ERR_ALLOC, "sliced layout: hipMalloc") : PSK_OK;
    }
    PSK_HIP(hipMemcpyAsync(A->sl_off, off.data(), (size_t)(nt + 1) * 8, hipMemcpyHostToDevice, s));
    PSK_HIP(hipMemcpyAsync(A->sl_woff, woff.data(), (size_t)(nt + 1) * 8, hipMemcpyHostToDevice, s));
    PSK_HIP(hipMemcpyAsync(A->sl_fmt, fmt.data(), (size_t)nt, hipMemcpyHostToDevice, s));
    if (!dict.empty()) {
        std::vector<double> padded(dict);
        padded.resize(kDictMax, 0.0);
        PSK_HIP(hipMemcpyAsync(A->sl_dict, padded.data(), kDictMax * 8, hipMemcpyHostToDevice, s));
    }
    A->sl_dict_n = (int32_t)dict.size();
    A->sl_uniform_w = uniform ? (int32_t)wmax : 0;
    A->sl_compact = compact ? 1 : 0;
    hipLaunchKernelGGL(sliced_fill_kernel, dim3((unsigned)nt), dim3(kBlock), 0, s, A->n, A->rowptr, A->colidx, A->vals,
                       A->sl_off, A->sl_woff, A->sl_fmt, A->sl_col, A->sl_pcol, A->sl_val, A->sl_dict,
                       A->sl_dict_n, compact ? 1 : 0);
    PSK_HIP(hipGetLastError());
    PSK_HIP(hipStreamSynchronize(s));
    A->sl_slots = slots;
    A->sl_packed_slots = packed_slots;
    A->sl_stream_bytes = stream;
    (void)wide_slots;
    return PSK_OK;
}

int csr_choose_layout(psk_csr *A, hipStream_t s) {
    const char *e = std::getenv("PSK_SPMV_LAYOUT");
    if (e && std::strcmp(e, "csr") == 0) return PSK_OK;
    // the diagonal layout first, when the matrix has one (it streams 1 B per row): automatically and with
    // PSK_SPMV_LAYOUT=diag (which otherwise falls back to the automatic choice); PSK_SPMV_DIAG=0 leaves it out
    const char *de = std::getenv("PSK_SPMV_DIAG");
    const bool diag_env = e && std::strcmp(e, "diag") == 0;
    if ((!e || diag_env) && !(de && std::atoi(de) == 0)) {
        PSK_TRY(diag_build(A, s, false));
        if (A->dg_mask) return PSK_OK;
    }
    if (diag_env) e = nullptr;
    const bool wide = e && std::strcmp(e, "sliced_wide") == 0;
    const bool plain = e && std::strcmp(e, "sliced") == 0;
    const bool force = e && (plain || wide || std::strcmp(e, "sliced_dict") == 0);
    // auto and sliced_dict: a dictionary when the values allow one (never an error here)
    int rc = sliced_build(A, s, force, !wide, !wide && !plain, false);
    if (rc != PSK_OK) sliced_free(A);
    return rc;
}

int tile_rows_for(int64_t n, int64_t nnz) {
    // rows per tile so that a typical tile's entries fit one LDS chunk
    const double avg = n > 0 ? (double)nnz / (double)n : 1.0;
    int r = kBlock;
    while (r > 32 && avg * r > kChunk) r >>= 1;
    return r;
}

// the dot of an SpMV over no rows: 0, into partial[0] and the mailbox like a finished grid sum
__global__ void spmv_empty_dot_kernel(GridSum gs, const int32_t *done) {
    if (threadIdx.x != 0 || (done && *done)) return;
    const double z[1] = {0.0};
    gs.out[0] = 0.0;
    gridsum_mail<1>(gs, z);
}

// the sliced and diagonal layouts' tiles in XCD bands (psk_internal.hpp; round 3)
static bool spmv_xcd_bands() { return true; }

// The CSR tile kernel's tile map (round 6): chunks of kCsrChunk consecutive tiles dealt over the
// XCDs (tile_map_chunked), so the +-m x lines a tile gathers were fetched through the same L2 by its chunk's
// neighbours; in the loop at N = 10M 0.1400 -> 0.1380 ms, back to back 0.1342 -> 0.1292 ms (block order: the x
// line neighbours land on other XCDs; the whole-band map measured 0.145 ms; profiles/r6_csr_tilemap_ab.txt).
// (-DPSK_CSR_CHUNK=0 builds block order.)
#ifndef PSK_CSR_CHUNK
#define PSK_CSR_CHUNK 128
#endif
static int64_t spmv_csr_chunk() { return PSK_CSR_CHUNK; }

// the pair-row diagonal kernel's half-slices per wave (round 6: 2 — a wave per slice; 1 measured slower, 0 = the
// one-row kernel: profiles/r6_diag_pair_ab.txt; -DPSK_DIAG_PAIR=0/1 builds the others)
#ifndef PSK_DIAG_PAIR
#define PSK_DIAG_PAIR 2
#endif
static int diag_pair_h() { return PSK_DIAG_PAIR; }
// slices per workgroup of the compact uniform sliced kernel (round 4: 2)
static int spmv_tpw() { return 2; }

static int64_t spmv_tiles(const psk_csr *A) { return (A->n + A->tile_rows - 1) / A->tile_rows; }

int launch_spmv(const psk_csr *A, int mode, const double *x, double *y, const double *aux_d,
                const double *aux_q, double *partial, const int32_t *done_flag, hipStream_t s, hipEvent_t ev0,
                hipEvent_t ev1, int rev, uint64_t *mail_seq) {
    Context *c;
    PSK_TRY(ctx(&c));
    const bool sliced = A->sl_off != nullptr || A->dg_mask != nullptr;   // 256-row slices
    const int64_t nwg = sliced ? (A->n + kSlice - 1) / kSlice : spmv_tiles(A);
    GridSum gs{nullptr, nullptr, nullptr, nullptr, 0, 0, -1, nullptr, nullptr, 0, 0};
    if (partial && nwg > 0) PSK_TRY(gridsum_prepare(c, nwg, 1, partial, &gs));
    if (partial && nwg == 0) gs.out = partial;
    if (mail_seq) {
        if (!partial || !A->comm || !A->comm->mb) return fail(PSK_ERR_ARG, "launch_spmv: mailbox without a dot");
        *mail_seq = mbox_next(A->comm, &gs);
    }
    if (A->n == 0) {   // no rows (an empty shard): the dot is 0, still published
        if (partial) {
            hipLaunchKernelGGL(spmv_empty_dot_kernel, dim3(1), dim3(64), 0, s, gs, done_flag);
            PSK_HIP(hipGetLastError());
        }
        return PSK_OK;
    }
    dim3 gd((unsigned)nwg), bd(kBlock);
    // XCD bands for the sliced layouts (N = 10M in the loop 0.078 -> 0.072 ms, back to back 0.067 ->
    // 0.057 ms); the CSR tile kernel measured 2-3% slower with them (3163^2 and 16384^2), so it keeps
    // block order
    // rev: each XCD walks its band backwards (the PCG loop alternates directions, PSK_K23_BANDS=2)
    TileMap tm = tile_map_for(nwg, sliced && spmv_xcd_bands(), rev != 0);
    if (!sliced && spmv_csr_chunk() > 0) tm = tile_map_chunked(nwg, spmv_csr_chunk());
    // compact uniform layout (FD and other 2-value stencils): slices per workgroup,
    // spmv_uniform_multi_kernel (round 4: 2 by default, PSK_SPMV_TPW=1 the one-slice kernel, 3 and 4
    // lab). Two slices per workgroup: in-loop SpMV at N = 10M 0.0657 -> 0.0611 ms, 16384^2 1.60 ->
    // 1.49 ms, same bits; with double values (the general path) it measured 4% slower and is not used
    // there (profiles/r4_spmv_ab.txt)
    const int tpw = spmv_tpw();
    const int64_t nwg2 = (nwg + tpw - 1) / tpw;
    const dim3 gd2((unsigned)(nwg2 > 0 ? nwg2 : 1));
    const TileMap tm2 = tile_map_for(nwg2, sliced && spmv_xcd_bands(), rev != 0);
    if (A->dg_mask) {   // diagonal layout: kDiagTpw slices per workgroup
        const DiagDesc dd = diag_desc(A);
        const int km = A->dg_K <= 3 ? 3 : A->dg_K <= 5 ? 5 : 8;
        const int64_t nwgd = (nwg + kDiagTpw - 1) / kDiagTpw;
        const dim3 gdd((unsigned)(nwgd > 0 ? nwgd : 1));
        const TileMap tmd = tile_map_for(nwgd, spmv_xcd_bands(), rev != 0);
        // the DPP neighbour form (PSK_DIAG_DPP builds) for the two 5-diagonal orders it is written for
        const int nbk = !kDiagDpp || A->dg_K != 5 ? 0
                        : (A->dg_d[0] == 0 && A->dg_d[3] == -1 && A->dg_d[4] == 1) ? 1
                        : (A->dg_d[2] == 0 && A->dg_d[1] == -1 && A->dg_d[3] == 1) ? 2 : 0;
        // round 6: the pair-row kernel (16-B accesses) for the two DPP orders
        const int pairh = (nbk != 0 && A->n >= 2 && dd.ncols >= 2) ? diag_pair_h() : 0;
        const int64_t nwgp = pairh ? (nwg + (pairh == 2 ? 4 : 2) - 1) / (pairh == 2 ? 4 : 2) : 1;
        const dim3 gdp((unsigned)nwgp);
        const TileMap tmp = tile_map_for(nwgp, spmv_xcd_bands(), rev != 0);
#define PSK_DIAGP(M, NB, H)                                                                                        \
    hipExtLaunchKernelGGL((spmv_diagp_kernel<M, NB, H>), gdp, bd, 0, s, ev0, ev1, 0, A->n, A->dg_mask, dd, x, y, aux_d, \
                          aux_q, gs, done_flag, tmp, nwg)
#define PSK_DIAG_LAUNCH(M, KM)                                                                                     \
    do {                                                                                                           \
        if (KM == 5 && pairh == 2 && nbk == 1) PSK_DIAGP(M, 1, 2);                                                 \
        else if (KM == 5 && pairh == 2 && nbk == 2) PSK_DIAGP(M, 2, 2);                                            \
        else if (KM == 5 && pairh == 1 && nbk == 1) PSK_DIAGP(M, 1, 1);                                            \
        else if (KM == 5 && pairh == 1 && nbk == 2) PSK_DIAGP(M, 2, 1);                                            \
        else if (KM == 5 && nbk == 1)                                                                              \
            hipExtLaunchKernelGGL((spmv_diag_kernel<M, 5, kDiagTpw, 1>), gdd, bd, 0, s, ev0, ev1, 0, A->n, A->dg_mask, \
                                  dd, x, y, aux_d, aux_q, gs, done_flag, tmd, nwg);                                 \
        else if (KM == 5 && nbk == 2)                                                                              \
            hipExtLaunchKernelGGL((spmv_diag_kernel<M, 5, kDiagTpw, 2>), gdd, bd, 0, s, ev0, ev1, 0, A->n, A->dg_mask, \
                                  dd, x, y, aux_d, aux_q, gs, done_flag, tmd, nwg);                                 \
        else                                                                                                       \
            hipExtLaunchKernelGGL((spmv_diag_kernel<M, KM, kDiagTpw>), gdd, bd, 0, s, ev0, ev1, 0, A->n, A->dg_mask, dd, \
                                  x, y, aux_d, aux_q, gs, done_flag, tmd, nwg);                                     \
    } while (0)
#define PSK_DIAG_MODE(M)                                                                                           \
    do {                                                                                                           \
        if (km == 3) PSK_DIAG_LAUNCH(M, 3);                                                                        \
        else if (km == 5) PSK_DIAG_LAUNCH(M, 5);                                                                   \
        else PSK_DIAG_LAUNCH(M, 8);                                                                                \
    } while (0)
        switch (mode) {
        case kSpmvPlain: PSK_DIAG_MODE(kSpmvPlain); break;
        case kSpmvDot: PSK_DIAG_MODE(kSpmvDot); break;
        case kSpmvJacobiDot: PSK_DIAG_MODE(kSpmvJacobiDot); break;
        case kSpmvPlainDot: PSK_DIAG_MODE(kSpmvPlainDot); break;
        case kSpmvResid: PSK_DIAG_MODE(kSpmvResid); break;
        case kSpmvAdd: PSK_DIAG_MODE(kSpmvAdd); break;
        default:
            return fail(PSK_ERR_ARG, "unknown spmv mode");
        }
#undef PSK_DIAG_MODE
#undef PSK_DIAG_LAUNCH
#undef PSK_DIAGP
        PSK_HIP(hipGetLastError());
        return PSK_OK;
    }
    if (sliced) {
        const int dk = !A->sl_dict ? 0 : A->sl_dict_n <= 2 ? 2 : A->sl_dict_n <= 4 ? 4 : 8;
        const int uw = A->sl_uniform_w;   // 0, or the uniform width (<= kSliceRegs)
#define PSK_UNI_LAUNCH(M, DK, UW)                                                                              \
    hipExtLaunchKernelGGL((spmv_uniform_kernel<M, DK, UW>), gd, bd, 0, s, ev0, ev1, 0, A->n, A->sl_pcol, A->sl_val, A->sl_dict, \
                       x, y, aux_d, aux_q, gs, done_flag, tm)
#define PSK_SLICED_LAUNCH_DK(M, DK)                                                                            \
    do {                                                                                                       \
        switch (uw) {                                                                                          \
        case 0:                                                                                                \
            hipExtLaunchKernelGGL((spmv_sliced_kernel<M, DK>), gd, bd, 0, s, ev0, ev1, 0, A->n, A->sl_off, A->sl_woff,         \
                               A->sl_fmt, A->sl_col, A->sl_pcol, A->sl_val, A->sl_dict, x, y, aux_d, aux_q, gs, \
                               done_flag, tm);                                                                     \
            break;                                                                                             \
        case 1: PSK_UNI_LAUNCH(M, DK, 1); break;                                                               \
        case 2: PSK_UNI_LAUNCH(M, DK, 2); break;                                                               \
        case 3: PSK_UNI_LAUNCH(M, DK, 3); break;                                                               \
        case 4: PSK_UNI_LAUNCH(M, DK, 4); break;                                                               \
        case 5: PSK_UNI_LAUNCH(M, DK, 5); break;                                                               \
        case 6: PSK_UNI_LAUNCH(M, DK, 6); break;                                                               \
        case 7: PSK_UNI_LAUNCH(M, DK, 7); break;                                                               \
        default: PSK_UNI_LAUNCH(M, DK, 8); break;                                                              \
        }                                                                                                      \
    } while (0)
#define PSK_UNI_LAUNCH_C(M, UW)                                                                                \
    do {                                                                                                       \
        if (tpw == 2)                                                                                          \
            hipExtLaunchKernelGGL((spmv_uniform_multi_kernel<M, 2, UW, true, 2>), gd2, bd, 0, s, ev0, ev1, 0, A->n,   \
                                  A->sl_pcol, A->sl_val, A->sl_dict, x, y, aux_d, aux_q, gs, done_flag, tm2, nwg);  \
        else if (tpw == 3)                                                                                     \
            hipExtLaunchKernelGGL((spmv_uniform_multi_kernel<M, 2, UW, true, 3>), gd2, bd, 0, s, ev0, ev1, 0, A->n,   \
                                  A->sl_pcol, A->sl_val, A->sl_dict, x, y, aux_d, aux_q, gs, done_flag, tm2, nwg);  \
        else if (tpw == 4)                                                                                     \
            hipExtLaunchKernelGGL((spmv_uniform_multi_kernel<M, 2, UW, true, 4>), gd2, bd, 0, s, ev0, ev1, 0, A->n,   \
                                  A->sl_pcol, A->sl_val, A->sl_dict, x, y, aux_d, aux_q, gs, done_flag, tm2, nwg);  \
        else                                                                                                   \
            hipExtLaunchKernelGGL((spmv_uniform_kernel<M, 2, UW, true>), gd, bd, 0, s, ev0, ev1, 0, A->n, A->sl_pcol,  \
                                  A->sl_val, A->sl_dict, x, y, aux_d, aux_q, gs, done_flag, tm);                 \
    } while (0)
#define PSK_SLICED_LAUNCH(M)                                                                                   \
    do {                                                                                                       \
        if (A->sl_compact) {   /* uniform, odd width, 2-entry dictionary */                                    \
            if (uw == 1) PSK_UNI_LAUNCH_C(M, 1);                                                               \
            else if (uw == 3) PSK_UNI_LAUNCH_C(M, 3);                                                          \
            else if (uw == 5) PSK_UNI_LAUNCH_C(M, 5);                                                          \
            else PSK_UNI_LAUNCH_C(M, 7);                                                                       \
        } else if (dk == 0) PSK_SLICED_LAUNCH_DK(M, 0);                                                        \
        else if (dk == 2) PSK_SLICED_LAUNCH_DK(M, 2);                                                          \
        else if (dk == 4) PSK_SLICED_LAUNCH_DK(M, 4);                                                          \
        else PSK_SLICED_LAUNCH_DK(M, 8);                                                                       \
    } while (0)
        switch (mode) {
        case kSpmvPlain: PSK_SLICED_LAUNCH(kSpmvPlain); break;
        case kSpmvDot: PSK_SLICED_LAUNCH(kSpmvDot); break;
        case kSpmvJacobiDot: PSK_SLICED_LAUNCH(kSpmvJacobiDot); break;
        case kSpmvPlainDot: PSK_SLICED_LAUNCH(kSpmvPlainDot); break;
        case kSpmvResid: PSK_SLICED_LAUNCH(kSpmvResid); break;
        case kSpmvAdd: PSK_SLICED_LAUNCH(kSpmvAdd); break;
        default:
            return fail(PSK_ERR_ARG, "unknown spmv mode");
        }
#undef PSK_SLICED_LAUNCH
#undef PSK_SLICED_LAUNCH_DK
#undef PSK_UNI_LAUNCH
#undef PSK_UNI_LAUNCH_C
        PSK_HIP(hipGetLastError());
        return PSK_OK;
    }
    const int tr = A->tile_rows;
    const int32_t nz = (int32_t)A->nnz;
#define PSK_SPMV_LAUNCH(M)                                                                                  \
    hipExtLaunchKernelGGL(spmv_kernel<M>, gd, bd, 0, s, ev0, ev1, 0, A->n, tr, A->rowptr, A->colidx, A->vals, x, y, aux_d, \
                       aux_q, gs, done_flag, nz, tm)
    switch (mode) {
    case kSpmvPlain: PSK_SPMV_LAUNCH(kSpmvPlain); break;
    case kSpmvDot: PSK_SPMV_LAUNCH(kSpmvDot); break;
    case kSpmvJacobiDot: PSK_SPMV_LAUNCH(kSpmvJacobiDot); break;
    case kSpmvPlainDot: PSK_SPMV_LAUNCH(kSpmvPlainDot); break;
    case kSpmvResid: PSK_SPMV_LAUNCH(kSpmvResid); break;
    case kSpmvAdd: PSK_SPMV_LAUNCH(kSpmvAdd); break;
    default:
        return fail(PSK_ERR_ARG, "unknown spmv mode");
    }
#undef PSK_SPMV_LAUNCH
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

// the DPP neighbour order of a 5-diagonal layout (spmv_diag_kernel's NB): 1 FD stored, 2 sorted, 0 neither
static int diag_nb(const psk_csr *A) {
    if (!kDiagDpp || !A->dg_mask || A->dg_K != 5) return 0;
    if (A->dg_d[0] == 0 && A->dg_d[3] == -1 && A->dg_d[4] == 1) return 1;
    if (A->dg_d[2] == 0 && A->dg_d[1] == -1 && A->dg_d[3] == 1) return 2;
    return 0;
}

bool pcg_init_diag_eligible(const psk_csr *A) { return !A->comm && A->n > 0 && diag_nb(A) != 0; }

int launch_pcg_init_diag(const psk_csr *A, const double *b, double xs, double *p, double *Ap, double *out3,
                         const PcgInitFin &fin, hipStream_t s) {
    if (!pcg_init_diag_eligible(A)) return fail(PSK_ERR_ARG, "launch_pcg_init_diag: not eligible");
    Context *c;
    PSK_TRY(ctx(&c));
    const int64_t nwg = (A->n + kSlice - 1) / kSlice, nwgd = (nwg + kDiagTpw - 1) / kDiagTpw;
    GridSum gs;
    PSK_TRY(gridsum_prepare(c, nwg, 3, out3, &gs));
    const DiagDesc dd = diag_desc(A);
    const TileMap tmd = tile_map_for(nwgd, spmv_xcd_bands());
    if (diag_nb(A) == 1)
        hipLaunchKernelGGL(pcg_init_diag_kernel<1>, dim3((unsigned)nwgd), dim3(kBlock), 0, s, A->n, A->dg_mask, dd, b, xs,
                           p, Ap, gs, fin, tmd, nwg);
    else
        hipLaunchKernelGGL(pcg_init_diag_kernel<2>, dim3((unsigned)nwgd), dim3(kBlock), 0, s, A->n, A->dg_mask, dd, b, xs,
                           p, Ap, gs, fin, tmd, nwg);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

// ---------------------------------------------------------------------------------------------
// FDLaplacian2D on the device (examples/FDLaplacian2D.py:5-23). Row k = m*iy + ix stores
// [diag, -m, +m, -1, +1] minus absent neighbours; rowptr in closed form
//   rowptr[k] = 5k - min(k,m) - max(0,k-m(m-1)) - ceil(k/m) - floor(k/m).
// Rows [row_begin, row_end) of the global matrix; column c is written as col_of(c) where
// local = c - col_shift for owned columns and halo columns map after the owned block.
__device__ __forceinline__ int64_t fd_rowptr(int64_t m, int64_t k) {
    int64_t mk = k < m ? k : m;
    int64_t top = k - m * (m - 1);
    if (top < 0) top = 0;
    return 5 * k - mk - top - (k + m - 1) / m - k / m;
}

__global__ void fd2d_kernel(int64_t m, int64_t row_begin, int64_t row_end, double dval, double oval,
                            int32_t *rowptr, int32_t *colidx, double *vals, int64_t halo_lo_start,
                            int64_t n_own) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nloc = row_end - row_begin;
    if (i > nloc) return;
    const int64_t k = row_begin + i;
    const int64_t base = fd_rowptr(m, row_begin);
    const int64_t off = fd_rowptr(m, k) - base;
    rowptr[i] = (int32_t)off;
    if (i == nloc) return;
    const int64_t ix = k % m, iy = k / m;
    // local column of a global column c: owned -> c-row_begin; below -> halo_lo; above -> halo_hi
    auto lc = [&](int64_t c) -> int32_t {
        if (c >= row_begin && c < row_end) return (int32_t)(c - row_begin);
        if (c < row_begin) return (int32_t)(n_own + (c - halo_lo_start));
        return (int32_t)(n_own + (row_begin - halo_lo_start) + (c - row_end));
    };
    int64_t p = off;
    colidx[p] = lc(k);
    vals[p++] = dval;
    if (iy > 0) { colidx[p] = lc(k - m); vals[p++] = oval; }
    if (iy < m - 1) { colidx[p] = lc(k + m); vals[p++] = oval; }
    if (ix > 0) { colidx[p] = lc(k - 1); vals[p++] = oval; }
    if (ix < m - 1) { colidx[p] = lc(k + 1); vals[p++] = oval; }
}

int fd2d_fill(psk_csr *A, int64_t m, double a, double b, int64_t row_begin, int64_t row_end,
              int64_t halo_lo_start, hipStream_t s) {
    const double h = std::fabs(b - a) / (double)(m + 1);   // FDLaplacian2D.py:6
    const double dval = -4.0 / h / h;                       // :13
    const double oval = 1.0 / h / h;                        // :15-21
    const int64_t nloc = row_end - row_begin;
    const int64_t threads = nloc + 1;
    const int64_t blocks = (threads + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(fd2d_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, m, row_begin, row_end,
                       dval, oval, A->rowptr, A->colidx, A->vals, halo_lo_start, nloc);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

// diagonal (scipy csr_diagonal: sum of col==row entries in stored order) and its reciprocal
__global__ void jacobi_dinv_kernel(int64_t n, const int32_t *rowptr, const int32_t *colidx,
                                   const double *vals, double *dinv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double d = 0.0;
    for (int32_t jj = rowptr[i]; jj < rowptr[i + 1]; ++jj)
        if (colidx[jj] == (int32_t)i) d = d + vals[jj];
    dinv[i] = 1.0 / d;   // np.reciprocal
}

// ---------------------------------------------------------------------------------------------
// BLAS-1 (dot / nrm2 / axpy) for the standalone entry points
__global__ __launch_bounds__(kBlock) void dot_partial_kernel(int64_t n, const double *__restrict__ x,
                                                             const double *__restrict__ y,
                                                             double *__restrict__ part) {
    __shared__ double sh[kWaves];
    int64_t t0, t1;
    const int64_t ntiles = (n + kVecTile - 1) / kVecTile;
    block_range(ntiles, t0, t1);
    const int64_t i0 = t0 * kVecTile, i1 = (t1 * kVecTile < n) ? t1 * kVecTile : n;
    double acc = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) acc = fma(x[i], y[i], acc);
    const double s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(kBlock) void reduce_final_kernel(const double *part, int np, double *out,
                                                              int do_sqrt) {
    __shared__ double sh[kWaves];
    const double s = reduce_partials(part, np, 1, sh);
    if (threadIdx.x == 0) out[0] = do_sqrt ? sqrt(s) : s;
}

__global__ void axpy_kernel(int64_t n, double alpha, const double *__restrict__ x, double *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = y[i] + alpha * x[i];   // compiled with -ffp-contract=off: two roundings
}

__global__ void scale_kernel(int64_t n, const double *__restrict__ d, const double *__restrict__ v,
                             double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = d[i] * v[i];
}

int prec_apply_dev(const psk_prec *M, int64_t n, const double *v, double *out, hipStream_t s) {
    if (n == 0) return PSK_OK;
    if (!M || M->kind == PSK_PREC_IDENTITY) {
        PSK_HIP(hipMemcpyAsync(out, v, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
        return PSK_OK;
    }
    if (M->kind == PSK_PREC_JACOBI) {
        hipLaunchKernelGGL(scale_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n,
                           M->dinv, v, out);
        PSK_HIP(hipGetLastError());
        return PSK_OK;
    }
    if (M->kind == PSK_PREC_ILU) return ilu_apply(M, v, out, s);
    if (M->kind == PSK_PREC_AMG) return amg_apply(M, v, out, s);
    if (M->kind == PSK_PREC_DENSE) return dense_apply(M, v, out, s);
    return fail(PSK_ERR_UNSUPPORTED, "unknown preconditioner kind");
}

}  // namespace psk

using namespace psk;

static int csr_alloc(psk_csr *A, int64_t n, int64_t nnz) {
    hipError_t e;
    e = hipMalloc(&A->rowptr, (size_t)(n + 1) * sizeof(int32_t));
    if (e != hipSuccess) return fail(PSK_ERR_ALLOC, "hipMalloc rowptr");
    {   // at least one entry: the SpMV's clamped stream loads always read a valid address
        const size_t m = nnz > 0 ? (size_t)nnz : 1;
        e = hipMalloc(&A->colidx, m * sizeof(int32_t));
        if (e != hipSuccess) return fail(PSK_ERR_ALLOC, "hipMalloc colidx");
        e = hipMalloc(&A->vals, m * sizeof(double));
        if (e != hipSuccess) return fail(PSK_ERR_ALLOC, "hipMalloc vals");
        if (nnz == 0) {
            e = hipMemset(A->colidx, 0, sizeof(int32_t));
            if (e == hipSuccess) e = hipMemset(A->vals, 0, sizeof(double));
            if (e != hipSuccess) return fail(PSK_ERR_HIP, "hipMemset dummy entry");
        }
    }
    return PSK_OK;
}

static void csr_free(psk_csr *A) {
    if (A->rowptr) (void)hipFree(A->rowptr);
    if (A->colidx) (void)hipFree(A->colidx);
    if (A->vals) (void)hipFree(A->vals);
    A->rowptr = nullptr;
    A->colidx = nullptr;
    A->vals = nullptr;
    sliced_free(A);
    diag_free(A);
    A->ws.release();
    A->ws_small.release();
    A->sendbuf.release();
    if (A->pack_idx) (void)hipFree(A->pack_idx);
    A->pack_idx = nullptr;
    A->pack_count = 0;
    A->peers.clear();
}

extern "C" {

int psk_csr_create(int64_t n, int64_t nnz, const int32_t *rowptr, const int32_t *colidx,
                   const double *vals, int32_t loc, psk_csr **out) {
    return psk_csr_create_rect(n, n, nnz, rowptr, colidx, vals, loc, out);
}

int psk_csr_create_rect(int64_t n, int64_t ncols, int64_t nnz, const int32_t *rowptr, const int32_t *colidx,
                        const double *vals, int32_t loc, psk_csr **out) {
    if (!out || n < 0 || ncols < 0 || nnz < 0 || !rowptr || (nnz > 0 && (!colidx || !vals)))
        return fail(PSK_ERR_ARG, "psk_csr_create: bad arguments");
    if (nnz > kMaxNnz || n >= INT32_MAX || ncols >= INT32_MAX)
        return fail(PSK_ERR_UNSUPPORTED, "psk_csr_create: int32 CSR indices required (nnz < 2^31 - 1536)");
    if (loc == PSK_HOST) {
        // a malformed CSR would make the gather fault on the device: validate it here, O(nnz)
        if (rowptr[0] != 0 || rowptr[n] != nnz)
            return fail(PSK_ERR_ARG, "psk_csr_create: rowptr[0] must be 0 and rowptr[n] == nnz");
        for (int64_t i = 0; i < n; ++i)
            if (rowptr[i + 1] < rowptr[i]) return fail(PSK_ERR_ARG, "psk_csr_create: rowptr not monotone");
        for (int64_t j = 0; j < nnz; ++j)
            if (colidx[j] < 0 || colidx[j] >= ncols) return fail(PSK_ERR_ARG, "psk_csr_create: column index out of range");
    }
    Context *c;
    PSK_TRY(ctx(&c));
    psk_csr *A = new psk_csr();
    A->n = n;
    A->ncols = ncols;
    A->nnz = nnz;
    A->tile_rows = tile_rows_for(n, nnz);
    A->n_global = n;
    A->row_begin = 0;
    A->row_end = n;
    A->device = c->device;
    int rc = csr_alloc(A, n, nnz);
    if (rc != PSK_OK) {
        csr_free(A);
        delete A;
        return rc;
    }
    const hipMemcpyKind k = loc == PSK_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    hipError_t e = hipMemcpyAsync(A->rowptr, rowptr, (size_t)(n + 1) * sizeof(int32_t), k, c->stream);
    if (e == hipSuccess && nnz > 0)
        e = hipMemcpyAsync(A->colidx, colidx, (size_t)nnz * sizeof(int32_t), k, c->stream);
    if (e == hipSuccess && nnz > 0)
        e = hipMemcpyAsync(A->vals, vals, (size_t)nnz * sizeof(double), k, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        csr_free(A);
        delete A;
        return fail(PSK_ERR_HIP, std::string("psk_csr_create copy: ") + hipGetErrorString(e));
    }
    rc = csr_choose_layout(A, c->stream);
    if (rc != PSK_OK) {
        csr_free(A);
        delete A;
        return rc;
    }
    *out = A;
    return PSK_OK;
}

int psk_csr_create_fd2d(double a, double b, int64_t m, psk_csr **out) {
    if (!out || m < 1) return fail(PSK_ERR_ARG, "psk_csr_create_fd2d: m must be >= 1");
    const int64_t n = m * m;
    const int64_t nnz = (m == 1) ? 1 : 5 * n - 4 * m;
    if (nnz > kMaxNnz) return fail(PSK_ERR_UNSUPPORTED, "FD2D: nnz exceeds int32 CSR");
    Context *c;
    PSK_TRY(ctx(&c));
    psk_csr *A = new psk_csr();
    A->n = n;
    A->ncols = n;
    A->nnz = nnz;
    A->tile_rows = tile_rows_for(n, nnz);
    A->n_global = n;
    A->row_end = n;
    A->device = c->device;
    int rc = csr_alloc(A, n, nnz);
    if (rc == PSK_OK) rc = fd2d_fill(A, m, a, b, 0, n, 0, c->stream);
    if (rc == PSK_OK) {
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = fail(PSK_ERR_HIP, std::string("fd2d: ") + hipGetErrorString(e));
    }
    if (rc == PSK_OK) rc = csr_choose_layout(A, c->stream);
    if (rc != PSK_OK) {
        csr_free(A);
        delete A;
        return rc;
    }
    *out = A;
    return PSK_OK;
}

int psk_csr_info(const psk_csr *A, int64_t *n, int64_t *nnz) {
    if (!A) return fail(PSK_ERR_ARG, "NULL matrix");
    if (n) *n = A->n;
    if (nnz) *nnz = A->nnz;
    return PSK_OK;
}

int psk_csr_layout(psk_csr *A, int32_t set, int32_t *layout, int64_t *slots, int64_t *packed_slots,
                   int64_t *stream_bytes) {
    if (!A) return fail(PSK_ERR_ARG, "psk_csr_layout: NULL matrix");
    if (set != -1 && set != PSK_LAYOUT_CSR && set != PSK_LAYOUT_SLICED && set != PSK_LAYOUT_SLICED_WIDE &&
        set != PSK_LAYOUT_SLICED_DICT && set != PSK_LAYOUT_DIAG)
        return fail(PSK_ERR_ARG, "psk_csr_layout: set must be -1 or a PSK_LAYOUT_* value");
    if (set != -1) {
        Context *c;
        PSK_TRY(ctx(&c));
        PSK_HIP(hipStreamSynchronize(c->stream));   // queued launches may still read the old layout
        if (set == PSK_LAYOUT_CSR) {
            sliced_free(A);
            diag_free(A);
        } else if (set == PSK_LAYOUT_DIAG) {
            PSK_TRY(diag_build(A, c->stream, true));
        } else {
            PSK_TRY(sliced_build(A, c->stream, true, set != PSK_LAYOUT_SLICED_WIDE, set == PSK_LAYOUT_SLICED_DICT,
                                 set == PSK_LAYOUT_SLICED_DICT));
        }
    }
    if (layout)
        *layout = A->dg_mask                  ? PSK_LAYOUT_DIAG
                  : !A->sl_off                ? PSK_LAYOUT_CSR
                  : A->sl_dict                ? PSK_LAYOUT_SLICED_DICT
                  : A->sl_packed_slots == 0   ? PSK_LAYOUT_SLICED_WIDE
                                              : PSK_LAYOUT_SLICED;
    if (slots) *slots = A->dg_mask ? A->n * A->dg_K : A->sl_slots;
    if (packed_slots) *packed_slots = A->dg_mask ? 0 : A->sl_packed_slots;
    // the diagonal layout streams one presence byte per row (its K offsets and values are kernel arguments)
    if (stream_bytes)
        *stream_bytes = A->dg_mask ? A->n : A->sl_off ? A->sl_stream_bytes : 12 * A->nnz + 4 * (A->n + 1);
    return PSK_OK;
}

int psk_csr_download(const psk_csr *A, int32_t *rowptr, int32_t *colidx, double *vals) {
    if (!A) return fail(PSK_ERR_ARG, "NULL matrix");
    Context *c;
    PSK_TRY(ctx(&c));
    if (rowptr)
        PSK_HIP(hipMemcpyAsync(rowptr, A->rowptr, (size_t)(A->n + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    if (colidx && A->nnz)
        PSK_HIP(hipMemcpyAsync(colidx, A->colidx, (size_t)A->nnz * 4, hipMemcpyDeviceToHost, c->stream));
    if (vals && A->nnz)
        PSK_HIP(hipMemcpyAsync(vals, A->vals, (size_t)A->nnz * 8, hipMemcpyDeviceToHost, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

int psk_csr_destroy(psk_csr *A) {
    if (!A || lib_shut_down()) return PSK_OK;   // after psk_shutdown: reclaimed with the process
    csr_free(A);
    delete A;
    return PSK_OK;
}

int psk_spmv(const psk_csr *Ac, const double *x, double *y, int32_t loc) {
    if (!Ac || !x || !y) return fail(PSK_ERR_ARG, "psk_spmv: NULL argument");
    psk_csr *A = const_cast<psk_csr *>(Ac);
    Context *c;
    PSK_TRY(ctx(&c));
    const double *dx = x;
    double *dy = y;
    DevBuf tmp;
    if (loc == PSK_HOST || A->comm) {
        // stage into [owned | halo] x and y
        PSK_TRY(tmp.ensure((size_t)(A->ncols + A->n) * sizeof(double)));
        double *tx = tmp.as<double>();
        const bool dry = A->comm && A->comm->dry;   // caller passes [owned | halo]
        const int64_t nx = (A->comm && !dry) ? A->n : A->ncols;   // rectangular: x has ncols entries
        PSK_TRY(to_device_vec(x, loc, nx, tx, c->stream));
        if (A->comm) PSK_TRY(halo_exchange(A, tx, c->stream));
        dx = tx;
        dy = (loc == PSK_HOST) ? tx + A->ncols : y;
    }
    PSK_TRY(launch_spmv(A, kSpmvPlain, dx, dy, nullptr, nullptr, nullptr, nullptr, c->stream));
    if (loc == PSK_HOST) PSK_TRY(from_device_vec(dy, PSK_HOST, A->n, y, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    tmp.release();
    return PSK_OK;
}

int psk_spmv_timed(const psk_csr *A, const double *x, double *y, int32_t reps, double *avg_ms) {
    if (!A || !x || !y || reps < 1 || !avg_ms) return fail(PSK_ERR_ARG, "psk_spmv_timed: bad arguments");
    if (A->comm) return fail(PSK_ERR_UNSUPPORTED, "psk_spmv_timed: sharded matrix");
    Context *c;
    PSK_TRY(ctx(&c));
    hipEvent_t e0, e1;
    PSK_HIP(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));   // timing only (runtime.hip)
    PSK_HIP(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    constexpr int mode = kSpmvPlain;
    DevBuf part;
    if (mode == kSpmvDot) PSK_TRY(part.ensure(64));
    double *pp = mode == kSpmvDot ? part.as<double>() : nullptr;
    int rc = launch_spmv(A, mode, x, y, nullptr, nullptr, pp, nullptr, c->stream);   // warm
    if (rc == PSK_OK && hipEventRecord(e0, c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "event record");
    for (int r = 0; r < reps && rc == PSK_OK; ++r)
        rc = launch_spmv(A, mode, x, y, nullptr, nullptr, pp, nullptr, c->stream);
    if (rc == PSK_OK && hipEventRecord(e1, c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "event record");
    float ms = 0.f;
    if (rc == PSK_OK && hipEventSynchronize(e1) != hipSuccess) rc = fail(PSK_ERR_HIP, "event sync");
    if (rc == PSK_OK && hipEventElapsedTime(&ms, e0, e1) != hipSuccess) rc = fail(PSK_ERR_HIP, "event time");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (mode == kSpmvDot) (void)hipStreamSynchronize(c->stream);   // before `part` is freed
    part.release();
    if (rc == PSK_OK) *avg_ms = (double)ms / reps;
    return rc;
}

static int dot_impl(int64_t n, const double *x, const double *y, int32_t loc, double *out, bool nrm) {
    if (!out || n < 0 || !x || (!nrm && !y)) return fail(PSK_ERR_ARG, "psk_dot: bad arguments");
    Context *c;
    PSK_TRY(ctx(&c));
    DevBuf tmp;
    const int grid = grid_for_rows(c, n, kVecTile);
    PSK_TRY(tmp.ensure((size_t)(2 * n + kMaxGrid + 1) * sizeof(double)));
    double *dx = const_cast<double *>(x), *dy = const_cast<double *>(y);
    double *base = tmp.as<double>();
    if (loc == PSK_HOST) {
        dx = base;
        PSK_TRY(to_device_vec(x, loc, n, dx, c->stream));
        if (!nrm) {
            dy = base + n;
            PSK_TRY(to_device_vec(y, loc, n, dy, c->stream));
        }
    }
    if (nrm) dy = dx;
    double *part = base + 2 * n;
    double *res = part + kMaxGrid;
    hipLaunchKernelGGL(dot_partial_kernel, dim3(grid), dim3(kBlock), 0, c->stream, n, dx, dy, part);
    PSK_HIP(hipGetLastError());
    hipLaunchKernelGGL(reduce_final_kernel, dim3(1), dim3(kBlock), 0, c->stream, part, grid, res, nrm ? 1 : 0);
    PSK_HIP(hipGetLastError());
    PSK_HIP(hipMemcpyAsync(out, res, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    tmp.release();
    return PSK_OK;
}

int psk_dot(int64_t n, const double *x, const double *y, int32_t loc, double *out) {
    return dot_impl(n, x, y, loc, out, false);
}

int psk_nrm2(int64_t n, const double *x, int32_t loc, double *out) {
    return dot_impl(n, x, nullptr, loc, out, true);
}

int psk_axpy(int64_t n, double alpha, const double *x, double *y, int32_t loc) {
    if (n < 0 || !x || !y) return fail(PSK_ERR_ARG, "psk_axpy: bad arguments");
    if (n == 0) return PSK_OK;
    Context *c;
    PSK_TRY(ctx(&c));
    DevBuf tmp;
    const double *dx = x;
    double *dy = y;
    if (loc == PSK_HOST) {
        PSK_TRY(tmp.ensure((size_t)2 * n * sizeof(double)));
        double *b = tmp.as<double>();
        PSK_TRY(to_device_vec(x, loc, n, b, c->stream));
        PSK_TRY(to_device_vec(y, loc, n, b + n, c->stream));
        dx = b;
        dy = b + n;
    }
    hipLaunchKernelGGL(axpy_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       c->stream, n, alpha, dx, dy);
    PSK_HIP(hipGetLastError());
    if (loc == PSK_HOST) PSK_TRY(from_device_vec(dy, PSK_HOST, n, y, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

// flag = 1 when some v[i] differs from v[0] bit for bit
__global__ void differs_from_first_kernel(int64_t n, const double *__restrict__ v, int32_t *flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && __double_as_longlong(v[i]) != __double_as_longlong(v[0])) *flag = 1;
}

int psk_prec_create(const psk_csr *A, int32_t kind, psk_prec **out) {
    if (!A || !out) return fail(PSK_ERR_ARG, "psk_prec_create: NULL argument");
    if (kind != PSK_PREC_IDENTITY && kind != PSK_PREC_JACOBI)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_create: unknown preconditioner kind");
    Context *c;
    PSK_TRY(ctx(&c));
    psk_prec *M = new psk_prec();
    M->kind = kind;
    M->n = A->n;
    if (kind == PSK_PREC_JACOBI && A->n > 0) {
        hipError_t e = hipMalloc(&M->dinv, (size_t)A->n * sizeof(double));
        if (e != hipSuccess) {
            delete M;
            return fail(PSK_ERR_ALLOC, "hipMalloc dinv");
        }
        hipLaunchKernelGGL(jacobi_dinv_kernel, dim3((unsigned)((A->n + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, c->stream, A->n, A->rowptr, A->colidx, A->vals, M->dinv);
        e = hipGetLastError();
        // a constant diagonal (stencils) gives one DInv value: the PCG kernels then use the scalar
        int32_t *dflag = nullptr;
        if (e == hipSuccess) e = hipMalloc(&dflag, sizeof(int32_t));
        if (e == hipSuccess) e = hipMemsetAsync(dflag, 0, sizeof(int32_t), c->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(differs_from_first_kernel, dim3((unsigned)((A->n + kBlock - 1) / kBlock)), dim3(kBlock),
                               0, c->stream, A->n, M->dinv, dflag);
            e = hipGetLastError();
        }
        int32_t differs = 1;
        if (e == hipSuccess) e = hipMemcpyAsync(&differs, dflag, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(&M->dinv_value, M->dinv, sizeof(double), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (dflag) (void)hipFree(dflag);
        const char *ue = std::getenv("PSK_JACOBI_UNIFORM");
        M->dinv_uniform = e == hipSuccess && differs == 0 && !(ue && std::atoi(ue) == 0);
        if (e != hipSuccess) {
            (void)hipFree(M->dinv);
            delete M;
            return fail(PSK_ERR_HIP, std::string("jacobi: ") + hipGetErrorString(e));
        }
    }
    *out = M;
    return PSK_OK;
}

int psk_prec_jacobi_uniform(const psk_prec *M, int32_t *uniform, double *value) {
    if (!M || M->kind != PSK_PREC_JACOBI) return fail(PSK_ERR_ARG, "psk_prec_jacobi_uniform: not a Jacobi preconditioner");
    if (uniform) *uniform = M->dinv_uniform ? 1 : 0;
    if (value) *value = M->dinv_uniform ? M->dinv_value : 0.0;
    return PSK_OK;
}

int psk_prec_apply(const psk_prec *M, int64_t n, const double *v, double *outv, int32_t loc) {
    if (!M || !v || !outv || n != M->n) return fail(PSK_ERR_ARG, "psk_prec_apply: bad arguments");
    Context *c;
    PSK_TRY(ctx(&c));
    if (n == 0) return PSK_OK;
    if (M->kind == PSK_PREC_IDENTITY) {
        const hipMemcpyKind k = loc == PSK_HOST ? hipMemcpyHostToHost : hipMemcpyDeviceToDevice;
        if (v != outv) PSK_HIP(hipMemcpyAsync(outv, v, (size_t)n * 8, k, c->stream));
        PSK_HIP(hipStreamSynchronize(c->stream));
        return PSK_OK;
    }
    DevBuf tmp;
    struct Release {   // (DevBuf has no destructor: the staging buffer was leaked before round 5)
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{tmp};
    const double *dv = v;
    double *dout = outv;
    if (loc == PSK_HOST || v == outv) {
        PSK_TRY(tmp.ensure((size_t)2 * n * sizeof(double)));
        double *b = tmp.as<double>();
        PSK_TRY(to_device_vec(v, loc, n, b, c->stream));
        dv = b;
        dout = b + n;
    }
    PSK_TRY(prec_apply_dev(M, n, dv, dout, c->stream));
    if (prec_is_general(M)) PSK_TRY(prec_check_error(M, c->stream));
    if (dout != outv) PSK_TRY(from_device_vec(dout, loc, n, outv, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

int psk_prec_destroy(psk_prec *M) {
    if (!M || lib_shut_down()) return PSK_OK;   // after psk_shutdown: reclaimed with the process
    void *ptrs[] = {M->dinv, M->gather_in, M->gather_out, M->work, M->err};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    M->lo.release();
    M->up.release();
    if (M->amg) amg_free(M->amg);
    if (M->dense) dense_free(M->dense);
    delete M;
    return PSK_OK;
}

int psk_prec_info(const psk_prec *M, int32_t *kind, int64_t *n, int64_t *nnz_l, int64_t *nnz_u, int64_t *levels_l,
                  int64_t *levels_u) {
    if (!M) return fail(PSK_ERR_ARG, "psk_prec_info: NULL preconditioner");
    if (kind) *kind = M->kind;
    if (n) *n = M->n;
    if (nnz_l) *nnz_l = M->lo.nnz;
    if (nnz_u) *nnz_u = M->up.nnz;
    if (levels_l) *levels_l = M->lo.levels;
    if (levels_u) *levels_u = M->up.levels;
    return PSK_OK;
}

}  // extern "C"

