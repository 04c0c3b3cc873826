// shmcomm.hip — a host shared-memory transport for the sharded solvers (validation of the multi-rank
// path on ONE GPU; no reference counterpart).
//
// RCCL refuses two ranks on one device, so a box with one MI355X cannot run the sharded PCG with
// P > 1 through RCCL. This transport runs the same collectives — the halo exchange of p and the
// allgathers of the ranks' dot products — between P processes of one host through a POSIX shared
// memory segment, enqueued on libpsk's stream like the RCCL calls they replace:
//   D2H of what this rank contributes -> host function: barrier of the P ranks -> H2D of the result.
// Everything else (shards, kernels, rank-order sums, host poll schedule) is the production path.
// It is slow (two PCIe copies and a host barrier per collective) and is never used for timing.
//
// Segment layout: a header (barrier counter, error flag) then two parity buffers (consecutive
// collectives alternate, so a rank that runs ahead never overwrites data a slower rank has not
// copied out yet: it cannot pass the next barrier before that rank's H2D, which precedes the
// rank's next host function in stream order), each [P senders][P receivers][slot] bytes.
#include "psk_internal.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

namespace psk {

constexpr size_t kShmSlot = (size_t)4 << 20;   // bytes one rank may send one peer per collective
constexpr size_t kShmHeader = 4096;

struct ShmHeader {
    std::atomic<int64_t> arrived;   // total barrier arrivals, all ranks
    std::atomic<int32_t> error;     // a barrier timed out somewhere
    std::atomic<int32_t> attached;
};

struct ShmComm {
    std::string name;
    int P = 1, r = 0;
    size_t bytes = 0;
    char *base = nullptr;
    int64_t barriers = 0;   // barriers this rank has entered (host-function order = stream order)
    int64_t gen = 0;        // collectives enqueued (parity buffer selection)
    ShmHeader *hdr() const { return reinterpret_cast<ShmHeader *>(base); }
    // slot of (sender, receiver) in parity buffer par
    char *slot(int64_t par, int snd, int rcv) const {
        return base + kShmHeader + ((size_t)par * P * P + (size_t)snd * P + (size_t)rcv) * kShmSlot;
    }
};

static void shm_barrier(ShmComm *sc) {
    ShmHeader *h = sc->hdr();
    const int64_t target = (int64_t)sc->P * (++sc->barriers);
    h->arrived.fetch_add(1, std::memory_order_acq_rel);
    const auto t0 = std::chrono::steady_clock::now();
    while (h->arrived.load(std::memory_order_acquire) < target) {
        if (h->error.load(std::memory_order_relaxed)) return;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
            h->error.store(1);
            std::fprintf(stderr, "psk shm transport: barrier timed out (ranks issued different collectives)\n");
            return;
        }
        std::this_thread::yield();
    }
}

static void shm_barrier_fn(void *p) { shm_barrier(static_cast<ShmComm *>(p)); }

int shm_error(const psk_comm *c) {
    if (c && c->shm && c->shm->hdr()->error.load()) return fail(PSK_ERR_RCCL, "shm transport: a barrier timed out");
    return PSK_OK;
}

// The collectives below are stream-ordered like their RCCL counterparts.
int shm_allgather(psk_comm *c, const double *send, double *recv, int64_t count, hipStream_t s) {
    ShmComm *sc = c->shm;
    const size_t b = (size_t)count * 8;
    if (b > kShmSlot) return fail(PSK_ERR_UNSUPPORTED, "shm transport: allgather larger than a slot");
    const int64_t par = (sc->gen++) & 1;
    PSK_HIP(hipMemcpyAsync(sc->slot(par, sc->r, 0), send, b, hipMemcpyDeviceToHost, s));
    PSK_HIP(hipLaunchHostFunc(s, shm_barrier_fn, sc));
    for (int q = 0; q < sc->P; ++q)
        PSK_HIP(hipMemcpyAsync(recv + (size_t)q * count, sc->slot(par, q, 0), b, hipMemcpyHostToDevice, s));
    return PSK_OK;
}

// sends[k] (device, counts[k] doubles) to peers[k]; receives recv_counts[k] doubles from peers[k]
// into recvs[k]
int shm_exchange(psk_comm *c, int npeers, const int *peers, const double *const *sends, const int64_t *send_counts,
                 double *const *recvs, const int64_t *recv_counts, hipStream_t s) {
    ShmComm *sc = c->shm;
    const int64_t par = (sc->gen++) & 1;
    for (int k = 0; k < npeers; ++k) {
        if ((size_t)send_counts[k] * 8 > kShmSlot || (size_t)recv_counts[k] * 8 > kShmSlot)
            return fail(PSK_ERR_UNSUPPORTED, "shm transport: halo larger than a slot");
        if (send_counts[k] > 0)
            PSK_HIP(hipMemcpyAsync(sc->slot(par, sc->r, peers[k]), sends[k], (size_t)send_counts[k] * 8,
                                   hipMemcpyDeviceToHost, s));
    }
    PSK_HIP(hipLaunchHostFunc(s, shm_barrier_fn, sc));
    for (int k = 0; k < npeers; ++k)
        if (recv_counts[k] > 0)
            PSK_HIP(hipMemcpyAsync(recvs[k], sc->slot(par, peers[k], sc->r), (size_t)recv_counts[k] * 8,
                                   hipMemcpyHostToDevice, s));
    return PSK_OK;
}

// synchronous host-side allgather of `bytes` per rank (creation-time checks)
int shm_allgather_host(psk_comm *c, const void *mine, void *all, size_t bytes) {
    ShmComm *sc = c->shm;
    Context *cx;
    PSK_TRY(ctx(&cx));
    PSK_HIP(hipStreamSynchronize(cx->stream));   // queued barriers of this rank run first
    if (bytes > kShmSlot) return fail(PSK_ERR_UNSUPPORTED, "shm transport: allgather larger than a slot");
    const int64_t par = (sc->gen++) & 1;
    std::memcpy(sc->slot(par, sc->r, 0), mine, bytes);
    shm_barrier(sc);
    for (int q = 0; q < sc->P; ++q) std::memcpy(static_cast<char *>(all) + (size_t)q * bytes, sc->slot(par, q, 0), bytes);
    return shm_error(c);
}

int shm_exchange_host(psk_comm *c, int npeers, const int *peers, const void *const *sends, const size_t *send_bytes,
                      void *const *recvs, const size_t *recv_bytes) {
    ShmComm *sc = c->shm;
    Context *cx;
    PSK_TRY(ctx(&cx));
    PSK_HIP(hipStreamSynchronize(cx->stream));
    const int64_t par = (sc->gen++) & 1;
    for (int k = 0; k < npeers; ++k) {
        if (send_bytes[k] > kShmSlot || recv_bytes[k] > kShmSlot)
            return fail(PSK_ERR_UNSUPPORTED, "shm transport: exchange larger than a slot");
        if (send_bytes[k]) std::memcpy(sc->slot(par, sc->r, peers[k]), sends[k], send_bytes[k]);
    }
    shm_barrier(sc);
    for (int k = 0; k < npeers; ++k)
        if (recv_bytes[k]) std::memcpy(recvs[k], sc->slot(par, peers[k], sc->r), recv_bytes[k]);
    return shm_error(c);
}

void shm_close(psk_comm *c) {
    ShmComm *sc = c->shm;
    if (!sc) return;
    if (sc->base) {
        (void)hipHostUnregister(sc->base);
        munmap(sc->base, sc->bytes);
    }
    if (sc->r == 0) shm_unlink(sc->name.c_str());
    delete sc;
    c->shm = nullptr;
}

}  // namespace psk

using namespace psk;

extern "C" int psk_comm_init_host(int32_t nranks, int32_t rank, const char *name, psk_comm **out) {
    if (!out || !name || nranks < 1 || rank < 0 || rank >= nranks || name[0] != '/' || std::strlen(name) > 200)
        return fail(PSK_ERR_ARG, "psk_comm_init_host: bad arguments (name must start with '/')");
    ShmComm *sc = new ShmComm();
    sc->name = name;
    sc->P = nranks;
    sc->r = rank;
    sc->bytes = kShmHeader + 2 * (size_t)nranks * nranks * kShmSlot;
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        delete sc;
        return fail(PSK_ERR_ARG, std::string("psk_comm_init_host: shm_open ") + name);
    }
    struct stat st;
    if (fstat(fd, &st) == 0 && (size_t)st.st_size < sc->bytes && ftruncate(fd, (off_t)sc->bytes) != 0) {
        close(fd);
        delete sc;
        return fail(PSK_ERR_ALLOC, "psk_comm_init_host: ftruncate");
    }
    void *p = mmap(nullptr, sc->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete sc;
        return fail(PSK_ERR_ALLOC, "psk_comm_init_host: mmap");
    }
    sc->base = static_cast<char *>(p);
    if (hipHostRegister(sc->base, sc->bytes, hipHostRegisterDefault) != hipSuccess) {
        munmap(sc->base, sc->bytes);
        delete sc;
        return fail(PSK_ERR_HIP, "psk_comm_init_host: hipHostRegister of the shared segment");
    }
    psk_comm *c = new psk_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->shm = sc;
    if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
    // every rank attached before anyone uses the segment (the creator's zero-filled header counts)
    sc->hdr()->attached.fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    while (sc->hdr()->attached.load() < nranks) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
            shm_close(c);
            delete c;
            return fail(PSK_ERR_RCCL, "psk_comm_init_host: peers did not attach");
        }
        std::this_thread::yield();
    }
    *out = c;
    return PSK_OK;
}
