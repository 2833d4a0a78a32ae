/*
 * dsm_ensemble.c -- the multi-GPU driver of the ensemble simulator, in C:
 * one host thread per GPU, each with its own dsm_ctx and a contiguous shard of system ids
 * (GPU g simulates ids [g*n, (g+1)*n): weak scaling, the counter-based generator makes every
 * system's trace depend only on its id), and ONE collective: an RCCL all-reduce over xGMI of
 * the counters and of the per-system aggregate (dsm_group_*), plus a max of the timed span.
 * No Python and no torch: this is the reference-style host program around the C ABI (the
 * reference runs one OpenMP thread per node of ONE system, assignment.c:125-153; this runs
 * one thread per GPU of an ensemble of them).
 *
 *   dsm_ensemble [--gpus N] [--config random|hot|evict] [--systems n] [--steps K]
 *                [--warmup W] [--type-counts]
 *
 * --config picks BASELINE.json's workloads (C3 random: 1M systems per GPU, C4 hot: 1M,
 * C5 evict: 2M; 8 nodes, 4096 instructions per node, seed 1).  A step = one pass of the
 * transition kernels over the GPU's shard, traces resident in HBM (generated on the device
 * before warmup).  --type-counts adds a parity pass after the timed steps with per-type
 * message counting (DSM_F_TYPE_COUNTS, the one-pass lock-step kernel) and reduces its
 * msgs_by_type too.  Prints one JSON line: per-rank aggregates, the job total, the reduced
 * counters and the rate; the caller checks them against tests/golden/aggregates.json
 * (<cfg>@r per shard, <cfg>@xN for the job).  Exit 0 on success, 1 on any error.
 */
#include <hip/hip_runtime_api.h>

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dsm.h"

#define MAX_GPUS 16
#define NP 8
#define N_INSTR 4096

typedef struct {
    const char *name;
    int dist;
    uint64_t systems;
    const char *workload;
} config_t;

static const config_t CONFIGS[] = {
    {"random", DSM_DIST_UNIFORM, 1u << 20,
     "C3: 1M synthetic 8-node systems/GPU, uniform RD/WR over 0x00-0x7F, 4096 instr/core"},
    {"hot", DSM_DIST_HOT, 1u << 20,
     "C4: 1M hot-line 8-node systems/GPU, RD/WR over {0x00,0x11,0x22,0x33}, 4096 instr/core"},
    {"evict", DSM_DIST_EVICT, 2u << 20,
     "C5: 2M eviction-heavy 8-node systems/GPU, {a: a%4==0}, 4096 instr/core"},
};

typedef struct {
    int rank, device, ngpus;
    const config_t *cfg;
    uint64_t n, first;
    int steps, warmup, type_counts;
    int syncs;                  /* sync_ok calls made */
    dsm_group *group;
    pthread_barrier_t *bar;
    volatile int *failed;
    /* results */
    int rc;
    const char *where;
    double elapsed_s;           /* this rank's timed span */
    uint64_t span_ns;           /* ... in ns, the all-reduce's input */
    uint64_t span_max_ns;       /* max over ranks (all-reduced) */
    dsm_aggregate local, total;
    dsm_counters counters_local, counters_total, types_total;
    float kms[64];
    uint32_t nkms;
} worker_t;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

#define CK(call, what) do { int e_ = (call); if (e_ != DSM_OK) { w->rc = e_; w->where = what; goto fail; } } while (0)
#define HK(call, what) do { if ((call) != hipSuccess) { w->rc = DSM_E_DEVICE; w->where = what; goto fail; } } while (0)

/* a host barrier that also tells every thread whether some thread failed: collectives are
 * entered only when all ranks got there (a rank that failed would leave the others blocked
 * inside RCCL) */
#define N_SYNC 2   /* host sync points of a worker (sync_ok calls) */
static int sync_ok(worker_t *w) {
    w->syncs++;
    pthread_barrier_wait(w->bar);
    const int ok = !*w->failed;
    pthread_barrier_wait(w->bar);
    return ok;
}

static void *worker(void *arg) {
    worker_t *w = (worker_t *)arg;
    dsm_ctx *ctx = NULL, *tctx = NULL;
    hipStream_t st = NULL;
    uint16_t *d_tr = NULL;
    uint32_t *d_cn = NULL;
    dsm_sys_result *d_res = NULL;
    dsm_counters *d_cnt = NULL, *d_tc = NULL;
    dsm_aggregate *d_agg = NULL;
    uint64_t *d_span = NULL;
    w->rc = DSM_OK;
    w->where = "";
    HK(hipSetDevice(w->device), "hipSetDevice");
    const dsm_config cfg = {NP, N_INSTR, 0, DSM_F_TIMING};
    CK(dsm_open(w->device, &cfg, &ctx), "dsm_open");
    HK(hipStreamCreate(&st), "hipStreamCreate");
    HK(hipMalloc((void **)&d_tr, w->n * NP * N_INSTR * sizeof(uint16_t)), "hipMalloc traces");
    HK(hipMalloc((void **)&d_cn, w->n * NP * sizeof(uint32_t)), "hipMalloc counts");
    HK(hipMalloc((void **)&d_res, w->n * sizeof(dsm_sys_result)), "hipMalloc results");
    HK(hipMalloc((void **)&d_cnt, sizeof(dsm_counters)), "hipMalloc counters");
    HK(hipMalloc((void **)&d_tc, sizeof(dsm_counters)), "hipMalloc type counters");
    HK(hipMalloc((void **)&d_agg, sizeof(dsm_aggregate)), "hipMalloc aggregate");
    HK(hipMalloc((void **)&d_span, sizeof(uint64_t)), "hipMalloc span");
    const dsm_gen gen = {1, w->cfg->dist, N_INSTR};
    CK(dsm_generate_device(ctx, &gen, w->first, w->n, d_tr, d_cn, st), "dsm_generate_device");
    for (int i = 0; i < w->warmup; ++i) {
        HK(hipMemsetAsync(d_cnt, 0, sizeof(dsm_counters), st), "hipMemsetAsync");
        CK(dsm_run_packed_device(ctx, d_tr, d_cn, w->n, d_res, d_cnt, st), "dsm_run_packed_device");
    }
    HK(hipStreamSynchronize(st), "warmup");
    if (!sync_ok(w)) goto done;
    /* timed region: a barrier over the GPUs (RCCL) on both sides, as bench.py */
    CK(dsm_group_barrier(w->group, st), "dsm_group_barrier");
    const double t0 = now_s();
    for (int i = 0; i < w->steps; ++i) {
        HK(hipMemsetAsync(d_cnt, 0, sizeof(dsm_counters), st), "hipMemsetAsync");
        CK(dsm_run_packed_device(ctx, d_tr, d_cn, w->n, d_res, d_cnt, st), "dsm_run_packed_device");
    }
    HK(hipStreamSynchronize(st), "steps");
    CK(dsm_group_barrier(w->group, st), "dsm_group_barrier");
    w->elapsed_s = now_s() - t0;
    CK(dsm_kernel_ms_history(ctx, w->kms, w->steps < 64 ? (uint32_t)w->steps : 64u, &w->nkms),
       "dsm_kernel_ms_history");

    /* the last step's results: this shard's aggregate on the device */
    HK(hipMemsetAsync(d_agg, 0, sizeof(dsm_aggregate), st), "hipMemsetAsync");
    CK(dsm_aggregate_device(ctx, d_res, w->n, w->first, d_agg, st), "dsm_aggregate_device");
    HK(hipMemcpyAsync(&w->local, d_agg, sizeof(dsm_aggregate), hipMemcpyDeviceToHost, st), "copy aggregate");
    HK(hipMemcpyAsync(&w->counters_local, d_cnt, sizeof(dsm_counters), hipMemcpyDeviceToHost, st), "copy counters");
    if (w->type_counts) {       /* parity pass: handled messages per transactionType */
        const dsm_config tcfg = {NP, N_INSTR, 0, DSM_F_TYPE_COUNTS};
        CK(dsm_open(w->device, &tcfg, &tctx), "dsm_open (type counts)");
        HK(hipMemsetAsync(d_tc, 0, sizeof(dsm_counters), st), "hipMemsetAsync");
        CK(dsm_run_packed_device(tctx, d_tr, d_cn, w->n, NULL, d_tc, st), "dsm_run_packed_device (type counts)");
    }
    HK(hipStreamSynchronize(st), "aggregate");
    if (!sync_ok(w)) goto done;
    /* the one collective: counters, aggregate (sums mod 2^64, a max), the timed span (max) */
    w->span_ns = (uint64_t)(w->elapsed_s * 1e9);
    HK(hipMemcpyAsync(d_span, &w->span_ns, sizeof w->span_ns, hipMemcpyHostToDevice, st), "copy span");
    CK(dsm_group_allreduce_counters(w->group, d_cnt, st), "dsm_group_allreduce_counters");
    CK(dsm_group_allreduce_aggregate(w->group, d_agg, st), "dsm_group_allreduce_aggregate");
    CK(dsm_group_allreduce(w->group, d_span, 1, DSM_RED_MAX, st), "dsm_group_allreduce");
    if (w->type_counts) CK(dsm_group_allreduce_counters(w->group, d_tc, st), "dsm_group_allreduce_counters");
    HK(hipMemcpyAsync(&w->counters_total, d_cnt, sizeof(dsm_counters), hipMemcpyDeviceToHost, st), "copy");
    HK(hipMemcpyAsync(&w->total, d_agg, sizeof(dsm_aggregate), hipMemcpyDeviceToHost, st), "copy");
    HK(hipMemcpyAsync(&w->span_max_ns, d_span, sizeof(uint64_t), hipMemcpyDeviceToHost, st), "copy");
    if (w->type_counts)
        HK(hipMemcpyAsync(&w->types_total, d_tc, sizeof(dsm_counters), hipMemcpyDeviceToHost, st), "copy");
    HK(hipStreamSynchronize(st), "reduce");
    goto done;
fail:
    *w->failed = 1;
    /* meet the host sync points this thread has not reached, so no thread waits for it (and
     * none enters a collective this rank will not join) */
    while (w->syncs < N_SYNC) sync_ok(w);
done:
    if (tctx) dsm_close(tctx);
    if (d_tr) hipFree(d_tr);
    if (d_cn) hipFree(d_cn);
    if (d_res) hipFree(d_res);
    if (d_cnt) hipFree(d_cnt);
    if (d_tc) hipFree(d_tc);
    if (d_agg) hipFree(d_agg);
    if (d_span) hipFree(d_span);
    if (st) hipStreamDestroy(st);
    if (ctx) dsm_close(ctx);
    return NULL;
}

static void print_agg(const dsm_aggregate *a) {
    printf("{\"systems\": %llu, \"msgs\": %llu, \"instrs\": %llu, \"rounds\": %llu, \"max_rounds\": %llu, "
           "\"status\": [%llu, %llu, %llu, %llu, %llu], \"sum_dump_hash\": \"0x%016llx\", "
           "\"sum_final_hash\": \"0x%016llx\", \"result_digest\": \"0x%016llx\"}",
           (unsigned long long)a->systems, (unsigned long long)a->msgs, (unsigned long long)a->instrs,
           (unsigned long long)a->rounds, (unsigned long long)a->max_rounds,
           (unsigned long long)a->by_status[0], (unsigned long long)a->by_status[1],
           (unsigned long long)a->by_status[2], (unsigned long long)a->by_status[3],
           (unsigned long long)a->by_status[4], (unsigned long long)a->sum_dump_hash,
           (unsigned long long)a->sum_final_hash, (unsigned long long)a->result_digest);
}

static int usage(void) {
    fprintf(stderr, "usage: dsm_ensemble [--gpus N] [--config random|hot|evict] [--systems n] "
                    "[--steps K] [--warmup W] [--type-counts]\n");
    return 1;
}

int main(int argc, char **argv) {
    int ngpus = 1, steps = 5, warmup = 1, type_counts = 0;
    uint64_t systems = 0;
    const config_t *cfg = &CONFIGS[0];
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "--gpus") && v) { ngpus = atoi(v); ++i; }
        else if (!strcmp(a, "--steps") && v) { steps = atoi(v); ++i; }
        else if (!strcmp(a, "--warmup") && v) { warmup = atoi(v); ++i; }
        else if (!strcmp(a, "--systems") && v) { systems = strtoull(v, NULL, 0); ++i; }
        else if (!strcmp(a, "--type-counts")) type_counts = 1;
        else if (!strcmp(a, "--config") && v) {
            cfg = NULL;
            for (size_t k = 0; k < sizeof CONFIGS / sizeof CONFIGS[0]; ++k)
                if (!strcmp(v, CONFIGS[k].name)) cfg = &CONFIGS[k];
            if (!cfg) return usage();
            ++i;
        } else return usage();
    }
    int have = 0;
    if (dsm_device_count(&have) != DSM_OK || have < 1) {
        fprintf(stderr, "dsm_ensemble: no gfx950 device\n");
        return 1;
    }
    if (ngpus < 1 || ngpus > MAX_GPUS || ngpus > have || steps < 1 || steps > 64 || warmup < 0) {
        fprintf(stderr, "dsm_ensemble: bad --gpus/--steps/--warmup (%d device(s) visible)\n", have);
        return 1;
    }
    const uint64_t n = systems ? systems : cfg->systems;
    int devices[MAX_GPUS];
    dsm_group *groups[MAX_GPUS];
    for (int g = 0; g < ngpus; ++g) devices[g] = g;
    int rc = dsm_group_init_all(ngpus, devices, groups);
    if (rc != DSM_OK) {
        fprintf(stderr, "dsm_ensemble: dsm_group_init_all: %s\n", dsm_strerror(rc));
        return 1;
    }
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)ngpus);
    volatile int failed = 0;
    worker_t W[MAX_GPUS];
    pthread_t th[MAX_GPUS];
    memset(W, 0, sizeof W);
    for (int g = 0; g < ngpus; ++g) {
        W[g] = (worker_t){.rank = g, .device = g, .ngpus = ngpus, .cfg = cfg, .n = n,
                          .first = (uint64_t)g * n, .steps = steps, .warmup = warmup,
                          .type_counts = type_counts, .group = groups[g], .bar = &bar,
                          .failed = &failed};
        pthread_create(&th[g], NULL, worker, &W[g]);
    }
    for (int g = 0; g < ngpus; ++g) pthread_join(th[g], NULL);
    pthread_barrier_destroy(&bar);
    for (int g = 0; g < ngpus; ++g) dsm_group_close(groups[g]);
    for (int g = 0; g < ngpus; ++g)
        if (W[g].rc != DSM_OK) {
            fprintf(stderr, "dsm_ensemble: rank %d: %s: %s\n", g, W[g].where, dsm_strerror(W[g].rc));
            return 1;
        }
    const worker_t *w0 = &W[0];
    const double span = (double)w0->span_max_ns * 1e-9;
    printf("{\"driver\": \"dsm_ensemble (C, one host thread per GPU, RCCL all-reduce via dsm_group_*)\", "
           "\"metric\": \"simulated coherence transactions/sec (whole node)\", \"value\": %.1f, "
           "\"unit\": \"transactions/s\", \"n_gpus\": %d, \"steps\": %d, \"warmup\": %d, "
           "\"ms_per_step\": %.3f, \"scaling\": \"weak\", \"dtype\": \"u8\", "
           "\"config\": {\"name\": \"%s\", \"workload\": \"%s\", \"systems_per_gpu\": %llu, \"np\": %d, "
           "\"instr_per_node\": %d, \"parallelism\": \"ensemble-dp%d\"}, "
           "\"collective\": \"rccl ncclAllReduce over %d GPU(s): dsm_counters + dsm_aggregate (sum, max) + timed span (max)\", ",
           (double)w0->counters_total.msgs * steps / span, ngpus, steps, warmup, span / steps * 1e3,
           cfg->name, cfg->workload, (unsigned long long)n, NP, N_INSTR, ngpus, ngpus);
    printf("\"kernel_ms\": [");
    for (uint32_t i = 0; i < w0->nkms; ++i) printf("%s%.3f", i ? ", " : "", w0->kms[i]);
    printf("], \"ranks\": [");
    for (int g = 0; g < ngpus; ++g) {
        printf("%s{\"rank\": %d, \"device\": %d, \"first_sys\": %llu, \"systems\": %llu, \"elapsed_s\": %.6f, "
               "\"counters_msgs\": %llu, \"aggregate\": ", g ? ", " : "", g, W[g].device,
               (unsigned long long)W[g].first, (unsigned long long)W[g].n, W[g].elapsed_s,
               (unsigned long long)W[g].counters_local.msgs);
        print_agg(&W[g].local);
        printf("}");
    }
    printf("], \"total\": ");
    print_agg(&w0->total);
    const dsm_counters *c = &w0->counters_total;
    printf(", \"counters\": {\"msgs\": %llu, \"instrs\": %llu, \"rounds\": %llu, \"systems\": %llu, "
           "\"max_rounds\": %llu, \"sum_dump_hash\": \"0x%016llx\", \"sum_final_hash\": \"0x%016llx\", "
           "\"overflow_reruns\": %llu, \"resumed\": %llu}",
           (unsigned long long)c->msgs, (unsigned long long)c->instrs, (unsigned long long)c->rounds,
           (unsigned long long)c->systems, (unsigned long long)c->max_rounds,
           (unsigned long long)c->sum_dump_hash, (unsigned long long)c->sum_final_hash,
           (unsigned long long)c->overflow_reruns, (unsigned long long)c->resumed);
    if (type_counts) {
        printf(", \"msgs_by_type\": [");
        for (int t = 0; t < DSM_NTYPES; ++t)
            printf("%s%llu", t ? ", " : "", (unsigned long long)w0->types_total.msgs_by_type[t]);
        printf("], \"type_pass_msgs\": %llu", (unsigned long long)w0->types_total.msgs);
    }
    printf("}\n");
    return 0;
}
