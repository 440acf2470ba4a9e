// comm.cpp — a stand-alone RCCL communicator (spai_comm_*): one rank per GPU,
// the xGMI path of the multi-GPU bench.
//
// The reference's multi-worker fan-out (main.rs:169-186,220-234) has no
// collective: each worker owns its Mcts + Model and plays its own games.  The
// sharded self-play bench (bench.py --gpus N) therefore needs no data-path
// collective either; it reduces its per-rank work counters (sims, games,
// evaluations, positions) and step times through this communicator once per
// run, beside the host group, so an N-GPU run proves that RCCL formed an
// N-rank communicator over the devices it ran on.  The learner's gradient
// all-reduce (learner.hip) is the path's one real exchange step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <cstdlib>
#include <thread>

#include "spai_internal.h"

// Every RCCL call here is non-blocking (ncclConfig_t.blocking = 0) and waited for
// with a bound (SPAI_COMM_TIMEOUT_S, default 120 s): a rank whose peer failed or never
// arrived gets SPAI_ERR_DEVICE back (the communicator aborted) instead of blocking
// forever inside ncclCommInitRank or a collective, so the caller can agree with the
// other ranks over its host group and go on without RCCL.
static double comm_timeout_s() {
    const char *v = std::getenv("SPAI_COMM_TIMEOUT_S");
    const double t = v ? std::atof(v) : 120.0;
    return t > 0 ? t : 120.0;
}

struct spai_comm {
    int device = 0;
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    spai::DevBuf<double> buf;
};

namespace spai {

// wait (bounded) until the communicator's pending operation leaves ncclInProgress
static ncclResult_t comm_wait(ncclComm_t comm, double seconds) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(comm, &st);
        if (r != ncclSuccess) return r;
        if (st != ncclInProgress) return st;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

void comm_destroy(spai_comm *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    c->buf.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int comm_create(int device, int rank, int world, const uint8_t *id, spai_comm **out) {
    *out = nullptr;
    SPAI_CHECK(world >= 1 && rank >= 0 && rank < world, SPAI_ERR_INVALID, "bad rank %d / world %d", rank, world);
    int ndev = 0;
    SPAI_HIP(hipGetDeviceCount(&ndev));
    SPAI_CHECK(device >= 0 && device < ndev, SPAI_ERR_INVALID, "device %d of %d", device, ndev);
    spai_comm *c = new spai_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    auto fail = [&](int rc) {
        comm_destroy(c);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("comm: device %d stream creation failed", device);
        return fail(SPAI_ERR_DEVICE);
    }
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == SPAI_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(uid.internal, id, SPAI_COMM_ID_BYTES);
    ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
    config.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, world, uid, rank, &config);
    if (r == ncclInProgress || (r == ncclSuccess && c->comm)) r = comm_wait(c->comm, comm_timeout_s());
    if (r != ncclSuccess) {
        if (c->comm) (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        set_error("ncclCommInitRank(world %d, rank %d, device %d) failed: %s", world, rank, device,
                  r == ncclInProgress ? "timed out (a peer failed or never arrived)" : ncclGetErrorString(r));
        return fail(SPAI_ERR_DEVICE);
    }
    int nr = 0;
    if (ncclCommCount(c->comm, &nr) != ncclSuccess || nr != world) {
        set_error("RCCL communicator reports %d ranks, expected %d", nr, world);
        return fail(SPAI_ERR_DEVICE);
    }
    *out = c;
    return SPAI_OK;
}

// n doubles of host memory reduced over the ranks (sum or max) in place: H2D,
// ncclAllReduce over xGMI, D2H, on the communicator's own stream
int comm_allreduce_f64(spai_comm *c, double *host, size_t n, int op) {
    SPAI_CHECK(op == SPAI_REDUCE_SUM || op == SPAI_REDUCE_MAX, SPAI_ERR_INVALID, "reduce op %d", op);
    if (n == 0) return SPAI_OK;
    SPAI_CHECK(c->comm, SPAI_ERR_DEVICE, "the communicator was aborted by an earlier failure");
    SPAI_HIP(hipSetDevice(c->device));
    if (c->buf.n < n) SPAI_TRY(c->buf.alloc(n));
    SPAI_HIP(hipMemcpyAsync(c->buf.p, host, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllReduce(c->buf.p, c->buf.p, n, ncclFloat64, op == SPAI_REDUCE_SUM ? ncclSum : ncclMax,
                                   c->comm, c->stream);
    if (r == ncclInProgress) r = comm_wait(c->comm, comm_timeout_s());
    SPAI_HIP(hipMemcpyAsync(host, c->buf.p, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    // the collective runs on the stream: wait for it with the same bound
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q = hipErrorNotReady;
    while (r == ncclSuccess && (q = hipStreamQuery(c->stream)) == hipErrorNotReady) {
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(c->comm, &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) r = st;
        else if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > comm_timeout_s())
            r = ncclInProgress;
        else std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (r != ncclSuccess) {   // abort: the stream's collective can then return; the communicator is unusable
        (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        set_error("ncclAllReduce of %zu doubles failed: %s", n,
                  r == ncclInProgress ? "timed out (a peer failed or never arrived)" : ncclGetErrorString(r));
        return SPAI_ERR_DEVICE;
    }
    SPAI_CHECK(q == hipSuccess, SPAI_ERR_DEVICE, "comm stream: %s", hipGetErrorString(q));
    return SPAI_OK;
}

}  // namespace spai

extern "C" {

int spai_comm_create(int device, int rank, int world, const uint8_t *id, spai_comm **out) {
    if (!out || !id) {
        spai::set_error("null argument to spai_comm_create");
        return SPAI_ERR_INVALID;
    }
    return spai::comm_create(device, rank, world, id, out);
}

int spai_comm_allreduce_f64(spai_comm *c, double *buf, size_t n, int op) {
    if (!c || (!buf && n)) {
        spai::set_error("null argument to spai_comm_allreduce_f64");
        return SPAI_ERR_INVALID;
    }
    return spai::comm_allreduce_f64(c, buf, n, op);
}

int spai_comm_info(spai_comm *c, int *rank, int *world, int *device) {
    if (!c) {
        spai::set_error("null communicator");
        return SPAI_ERR_INVALID;
    }
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    if (device) *device = c->device;
    return SPAI_OK;
}

int spai_comm_destroy(spai_comm *c) {
    spai::comm_destroy(c);
    return SPAI_OK;
}

}  // extern "C"
