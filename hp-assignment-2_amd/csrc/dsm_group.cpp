/*
 * dsm_group.cpp -- the multi-GPU group of libdsm.so (include/dsm.h, dsm_group_*): one RCCL
 * communicator per GPU, over xGMI, for the ONE collective the ensemble needs:
 * the end-of-run all-reduce of the counters (dsm_counters, 320 B) and of the per-system
 * aggregate (dsm_aggregate, 128 B).  Systems are independent, so there is no data-path
 * exchange at all; the reductions are a few hundred bytes, latency-bound, and each is one
 * ncclAllReduce of uint64 (mod 2^64 sums) plus one single-slot max.
 *
 * The reference (assignment.c) has no multi-GPU side: its only sharing is sendMessage's
 * per-node queues (:711-739), which here stay inside a wavefront (dsm_engine.hip).
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdlib.h>
#include <string.h>

#include "dsm.h"

struct dsm_group {
    ncclComm_t comm;
    int rank, nranks, device;
    uint64_t *d_tmp;            /* one slot: the max-reduced value during a mixed reduction */
};

namespace {

int nck(ncclResult_t r) { return r == ncclSuccess ? DSM_OK : DSM_E_DEVICE; }
#define NCK(x) do { const int e_ = nck(x); if (e_) return e_; } while (0)
#define HCK(x) do { if ((x) != hipSuccess) return DSM_E_DEVICE; } while (0)

int new_group(ncclComm_t comm, int rank, int nranks, int device, dsm_group **out) {
    dsm_group *g = static_cast<dsm_group *>(calloc(1, sizeof(dsm_group)));
    if (!g) return DSM_E_NOMEM;
    g->comm = comm;
    g->rank = rank;
    g->nranks = nranks;
    g->device = device;
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&g->d_tmp, sizeof(uint64_t)) != hipSuccess) {
        ncclCommDestroy(comm);
        free(g);
        return DSM_E_DEVICE;
    }
    *out = g;
    return DSM_OK;
}

/* every slot of d[0 .. n) summed across ranks, except slot mx (max); in place on `st` */
int sum_with_max(dsm_group *g, uint64_t *d, size_t n, size_t mx, hipStream_t st) {
    HCK(hipSetDevice(g->device));
    /* the max reads slot mx before the in-place sum overwrites it: two launches in stream
     * order on the same communicator (not fused in a group, whose order is not specified) */
    NCK(ncclAllReduce(d + mx, g->d_tmp, 1, ncclUint64, ncclMax, g->comm, st));
    NCK(ncclAllReduce(d, d, n, ncclUint64, ncclSum, g->comm, st));
    HCK(hipMemcpyAsync(d + mx, g->d_tmp, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    return DSM_OK;
}

}  // namespace

static_assert(sizeof(ncclUniqueId) == DSM_GROUP_ID_BYTES, "DSM_GROUP_ID_BYTES");
static_assert(sizeof(dsm_aggregate) == DSM_NAGG * 8, "dsm_aggregate size");
static_assert(offsetof(dsm_aggregate, max_rounds) == DSM_AGG_MAX_SLOT * 8, "DSM_AGG_MAX_SLOT");

extern "C" int dsm_group_unique_id(unsigned char id[DSM_GROUP_ID_BYTES]) {
    if (!id) return DSM_E_INVAL;
    ncclUniqueId u;
    NCK(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return DSM_OK;
}

extern "C" int dsm_group_init_rank(int device, int nranks, int rank,
                                   const unsigned char id[DSM_GROUP_ID_BYTES], dsm_group **group) {
    if (!id || !group || nranks < 1 || rank < 0 || rank >= nranks || device < 0) return DSM_E_INVAL;
    *group = nullptr;
    HCK(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclComm_t comm;
    NCK(ncclCommInitRank(&comm, nranks, u, rank));
    return new_group(comm, rank, nranks, device, group);
}

extern "C" int dsm_group_init_all(int ndev, const int *devices, dsm_group **groups) {
    if (ndev < 1 || !devices || !groups) return DSM_E_INVAL;
    ncclComm_t *comms = static_cast<ncclComm_t *>(calloc((size_t)ndev, sizeof(ncclComm_t)));
    if (!comms) return DSM_E_NOMEM;
    const int e = nck(ncclCommInitAll(comms, ndev, devices));
    if (e) {
        free(comms);
        return e;
    }
    int rc = DSM_OK;
    for (int i = 0; i < ndev; ++i) {
        groups[i] = nullptr;
        if (rc == DSM_OK) rc = new_group(comms[i], i, ndev, devices[i], &groups[i]);
        else ncclCommDestroy(comms[i]);
    }
    free(comms);
    if (rc != DSM_OK)
        for (int i = 0; i < ndev; ++i)
            if (groups[i]) { dsm_group_close(groups[i]); groups[i] = nullptr; }
    return rc;
}

extern "C" int dsm_group_info(const dsm_group *g, int *rank, int *nranks, int *device) {
    if (!g) return DSM_E_INVAL;
    if (rank) *rank = g->rank;
    if (nranks) *nranks = g->nranks;
    if (device) *device = g->device;
    return DSM_OK;
}

extern "C" int dsm_group_close(dsm_group *g) {
    if (!g) return DSM_OK;
    int rc = DSM_OK;
    if (hipSetDevice(g->device) != hipSuccess) rc = DSM_E_DEVICE;
    if (g->d_tmp) (void)hipFree(g->d_tmp);
    if (ncclCommDestroy(g->comm) != ncclSuccess) rc = DSM_E_DEVICE;
    free(g);
    return rc;
}

extern "C" int dsm_group_allreduce(dsm_group *g, uint64_t *d_buf, size_t n, int op, void *stream) {
    if (!g || (n && !d_buf) || (op != DSM_RED_SUM && op != DSM_RED_MAX)) return DSM_E_INVAL;
    if (n == 0) return DSM_OK;
    HCK(hipSetDevice(g->device));
    NCK(ncclAllReduce(d_buf, d_buf, n, ncclUint64, op == DSM_RED_SUM ? ncclSum : ncclMax, g->comm,
                      (hipStream_t)stream));
    return DSM_OK;
}

extern "C" int dsm_group_allreduce_counters(dsm_group *g, dsm_counters *d_counters, void *stream) {
    if (!g || !d_counters) return DSM_E_INVAL;
    return sum_with_max(g, reinterpret_cast<uint64_t *>(d_counters), DSM_NCOUNTERS,
                        offsetof(dsm_counters, max_rounds) / 8, (hipStream_t)stream);
}

extern "C" int dsm_group_allreduce_aggregate(dsm_group *g, dsm_aggregate *d_agg, void *stream) {
    if (!g || !d_agg) return DSM_E_INVAL;
    return sum_with_max(g, reinterpret_cast<uint64_t *>(d_agg), DSM_NAGG, DSM_AGG_MAX_SLOT,
                        (hipStream_t)stream);
}

extern "C" int dsm_group_barrier(dsm_group *g, void *stream) {
    if (!g) return DSM_E_INVAL;
    HCK(hipSetDevice(g->device));
    NCK(ncclAllReduce(g->d_tmp, g->d_tmp, 1, ncclUint64, ncclMax, g->comm, (hipStream_t)stream));
    HCK(hipStreamSynchronize((hipStream_t)stream));
    return DSM_OK;
}
