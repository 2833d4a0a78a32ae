/*
 * cache_simulator.c -- drop-in replacement for the reference's process contract
 * (ruubhagat/HP-Assignment-2, README.md:86-106, assignment.c:118-123):
 *
 *     ./cache_simulator <test_directory>
 *
 * reads tests/<test_directory>/core_<n>.txt relative to the CWD (:794) and scans them on the
 * GPU (initializeProcessor's fgets/sscanf semantics), prints "Processor <n> initialized" per
 * node (:821), simulates the system on the GPU through libdsm.so under the deterministic
 * lock-step schedule, and writes the printProcessorState dump core_<n>_output.txt
 * (:824-876) of every node that finished issuing into the CWD, formatted on the GPU.
 *
 * Unlike the reference (whose loop never exits, :153, :584-587) it exits once the system is
 * quiescent: 0 = every node dumped, 2 = deadlocked (the stuck nodes write no dump, as in the
 * reference), 3 = ring overflow / assert / round limit, 1 = usage or I/O error.
 *
 * Options (all optional; defaults reproduce the reference build):
 *   --np N           number of nodes, 4 (NUM_PROCS, :9) or 8
 *   --max-instr N    instructions read per core file, default 32 (MAX_INSTR_NUM, :13)
 *   --device D       GPU ordinal, default 0
 *   --quiet          do not print the "initialized" lines
 *   --issue-order F  write the issue order to file F in the reference's DEBUG_INSTR format
 *                    (:595-598), as the schedule issued the instructions
 *   --schedule S:T   seeded schedule exploration (dsm_set_schedule): seed S, act threshold T
 *                    (0..65536; 65536 = lock-step); samples the reference's interleavings
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsm.h"

static void usage(const char *argv0) {
    fprintf(stderr, "Usage: %s [--np 4|8] [--max-instr N] [--device D] [--quiet] [--issue-order FILE]\n"
                    "          [--schedule SEED:THRESH] <test_directory>\n", argv0);
}

int main(int argc, char **argv) {
    int np = 4, device = 0, quiet = 0;
    uint32_t max_instr = DSM_REF_MAX_INSTR;
    const char *dir = NULL, *issue_file = NULL;
    unsigned long long sched_seed = 0;
    unsigned sched_thresh = DSM_SCHED_LOCKSTEP;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--np") && i + 1 < argc) np = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--max-instr") && i + 1 < argc) max_instr = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--quiet")) quiet = 1;
        else if (!strcmp(argv[i], "--issue-order") && i + 1 < argc) issue_file = argv[++i];
        else if (!strcmp(argv[i], "--schedule") && i + 1 < argc) {
            if (sscanf(argv[++i], "%llu:%u", &sched_seed, &sched_thresh) != 2) { usage(argv[0]); return EXIT_FAILURE; }
        }
        else if (argv[i][0] == '-' && argv[i][1] == '-') { usage(argv[0]); return EXIT_FAILURE; }
        else dir = argv[i];
    }
    if (!dir) { usage(argv[0]); return EXIT_FAILURE; }                 /* :119-122 */
    if ((np != 4 && np != 8) || max_instr == 0 || max_instr > DSM_MAX_INSTR) {
        usage(argv[0]);
        return EXIT_FAILURE;
    }
    const uint32_t stride = (max_instr + 7u) & ~7u;
    /* initializeProcessor (:776-822): the core files are read from disk here and scanned on
     * the GPU with the reference's fgets/sscanf semantics (dsm_parse_traces) */
    char *text = NULL;
    uint64_t off[DSM_MAX_NP + 1] = {0};
    for (int n = 0; n < np; ++n) {
        char path[256];
        snprintf(path, sizeof path, "tests/%s/core_%d.txt", dir, n);   /* :794 */
        FILE *f = fopen(path, "rb");
        if (!f) {                                                      /* :796-800 */
            fprintf(stderr, "Error: could not open file %s\n", path);
            perror("fopen");
            exit(EXIT_FAILURE);
        }
        char buf[1 << 16];
        size_t k;
        uint64_t len = off[n];
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) {
            char *t = (char *)realloc(text, len + k);
            if (!t) { fclose(f); return EXIT_FAILURE; }
            text = t;
            memcpy(text + len, buf, k);
            len += k;
        }
        fclose(f);
        off[n + 1] = len;
    }
    dsm_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.np = np;
    cfg.max_instr = stride;
    cfg.flags = DSM_F_SNAPSHOTS | (issue_file ? DSM_F_ISSUE_TRACE : 0u);
    dsm_ctx *ctx = NULL;
    int rc = dsm_open(device, &cfg, &ctx);
    if (rc) {
        fprintf(stderr, "Error: dsm_open: %s\n", dsm_strerror(rc));
        return EXIT_FAILURE;
    }

    uint16_t *traces = (uint16_t *)calloc((size_t)np * stride, sizeof(uint16_t));
    uint32_t counts[DSM_MAX_NP] = {0};
    int32_t pst[DSM_MAX_NP] = {0};
    if (!traces) return EXIT_FAILURE;
    rc = dsm_parse_traces(ctx, text ? text : "", off, (uint64_t)np, max_instr, traces, counts, pst);
    if (rc) {
        fprintf(stderr, "Error: dsm_parse_traces: %s\n", dsm_strerror(rc));
        return EXIT_FAILURE;
    }
    for (int n = 0; n < np; ++n) {
        if (pst[n]) {
            fprintf(stderr, "Error: tests/%s/core_%d.txt: %s (instruction %u)\n", dir, n,
                    dsm_strerror(pst[n]), counts[n]);
            exit(EXIT_FAILURE);
        }
        if (!quiet) printf("Processor %d initialized\n", n);           /* :821 */
    }
    fflush(stdout);
    free(text);

    if ((rc = dsm_set_schedule(ctx, sched_seed, sched_thresh))) {
        fprintf(stderr, "Error: dsm_set_schedule: %s\n", dsm_strerror(rc));
        return EXIT_FAILURE;
    }
    dsm_sys_result res;
    rc = dsm_run_packed(ctx, traces, counts, 1, &res, NULL);
    if (rc) {
        fprintf(stderr, "Error: dsm_run_packed: %s\n", dsm_strerror(rc));
        dsm_close(ctx);
        return EXIT_FAILURE;
    }
    const uint32_t status = res.status & 0xFFu, dumped = res.status >> 8;
    if (issue_file) {                                   /* DEBUG_INSTR order, :595-598 */
        uint32_t n = 0, cap = (uint32_t)np * stride;
        uint32_t *ev = (uint32_t *)malloc(cap * sizeof(uint32_t));
        char *txt = (char *)malloc((size_t)cap * 64 + 1);
        FILE *f = NULL;
        if (!ev || !txt || (rc = dsm_get_issue_trace(ctx, 0, ev, cap, &n)) ||
            (rc = dsm_format_issue_trace(ev, n < cap ? n : cap, txt, (size_t)cap * 64 + 1)) < 0 ||
            !(f = fopen(issue_file, "w")) || fwrite(txt, 1, (size_t)rc, f) != (size_t)rc) {
            fprintf(stderr, "Error: issue order: %s\n", rc < 0 ? dsm_strerror(rc) : "write failed");
            dsm_close(ctx);
            return EXIT_FAILURE;
        }
        fclose(f);
        free(ev);
        free(txt);
    }
    /* printProcessorState of every node that finished issuing (:695), formatted on the GPU */
    if ((rc = dsm_write_run_dumps(ctx, 0, dumped, NULL))) {
        fprintf(stderr, "Error: dumps: %s\n", dsm_strerror(rc));
        dsm_close(ctx);
        return EXIT_FAILURE;
    }
    dsm_close(ctx);
    free(traces);
    if (status == DSM_COMPLETED) return 0;
    if (status == DSM_DEADLOCKED) return 2;
    return 3;
}
