/*
 * oracle/ref_lockstep.c -- TEST INFRASTRUCTURE ONLY.  Built into oracle/_ref/ by
 * oracle/build_ref.sh when /root/reference is present; never shipped, never linked into
 * the product.
 *
 * Drives the reference's OWN code (/root/reference/assignment.c) single-threaded under the
 * deterministic lock-step schedule.  build_ref.sh extracts these line
 * ranges into a scratch directory at build time (they never enter this repository):
 *   frag_types.inc    assignment.c:15-81   types (NUM_PROCS / MAX_INSTR_NUM given by -D)
 *   frag_helpers.inc  assignment.c:94-115  isBitSet / findOwner / countSharers
 *   frag_handler.inc  assignment.c:177-566 message decode + 13-way handler switch
 *   frag_issue.inc    assignment.c:590-697 instruction issue + dump-once block
 *   frag_repl.inc     assignment.c:742-773 handleCacheReplacement
 *   frag_init.inc     assignment.c:776-822 initializeProcessor
 *   frag_print.inc    assignment.c:824-876 printProcessorState
 * This file supplies only what replaces the OpenMP runtime: per-node contexts for the loop
 * locals of main (:137-146), a staging sendMessage (deliveries at the end of each round,
 * ascending sender then program order), the round loop, and a record/hash writer.
 *
 * Usage:
 *   ref_lockstep tests <name> <out.bin>      (CWD must contain tests/<name>/core_n.txt;
 *                                            dumps written to CWD by printProcessorState)
 *   ref_lockstep tests <name> <out.bin> <seed> <thresh> <first> <n>
 *                                            (n seeded schedule-exploration variants; no files)
 *   ref_lockstep gen <dist> <seed> <n_instr> <first_sys> <n_sys> <out.bin>
 *   ref_lockstep fmt <recs.bin> <out.bin>   (printProcessorState of 64-byte records)
 *   ref_lockstep bench <dist> <seed> <n_instr> <first> <n> <nproc>
 *                                            (CPU baseline: timed run_system, forked slices)
 *   ref_lockstep agg <dist> <seed> <n_instr> <first> <n> <nproc>
 *                                            (full-size golden aggregates, forked slices)
 * out.bin: per system one dsm_res, then NUM_PROCS dump records, then NUM_PROCS final records.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <ctype.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <stdint.h>
#include "dsm_common.h"

#ifndef NUM_PROCS
#error "NUM_PROCS must be given"
#endif
#define CACHE_SIZE 4
#define MEM_SIZE 16
#define MSG_BUFFER_SIZE 256

/* asserts of the regular build abort the process; here they end the system with
 * ST_ASSERT_FAILED at the end of the round (the enclosing handler returns at the failed
 * assert; the other nodes finish their actions of that round; nothing is delivered). */
static int g_assert_failed;
#define assert(e) do { if (!(e)) { g_assert_failed = 1; return; } } while (0)

#include "frag_types.inc"

void initializeProcessor(int threadId, processorNode *node, char *dirName);
void sendMessage(int receiver, message msg);
void handleCacheReplacement(int sender, cacheLine oldCacheLine);
void printProcessorState(int processorId, processorNode node);

#include "frag_helpers.inc"

#define MAX_STAGED 1024
static message st_msg[MAX_STAGED];
static int st_dest[MAX_STAGED];
static int nst;

void sendMessage(int receiver, message msg) {
    if (nst < MAX_STAGED) { st_dest[nst] = receiver; st_msg[nst] = msg; }
    nst++;
}

#include "frag_repl.inc"
#include "frag_init.inc"
#include "frag_print.inc"

typedef struct {
    processorNode node;
    message msgReply;
    instruction instr;
    int instructionIdx;
    int instructions_done;
    processorNode dumpSnap;
    int dumped;
    message ring[MSG_BUFFER_SIZE];
    int head, count;
} nodeCtx;

static nodeCtx C[NUM_PROCS];
static int g_write_files;

static void capture_dump(int id, processorNode n) {
    C[id].dumpSnap = n;
    C[id].dumped = 1;
    if (g_write_files) printProcessorState(id, n);
}

static void handle(int threadId, nodeCtx *c, message msg) {
#define node (c->node)
#define msgReply (c->msgReply)
#include "frag_handler.inc"
#undef node
#undef msgReply
}

static void issue(int threadId, nodeCtx *c) {
#define node (c->node)
#define instr (c->instr)
#define instructionIdx (c->instructionIdx)
#define instructions_done (c->instructions_done)
#define printProcessorState capture_dump
#include "frag_issue.inc"
#undef printProcessorState
#undef instructions_done
#undef instructionIdx
#undef instr
#undef node
}

static void to_rec(const processorNode *n, int waiting, int done, int issued, dsm_rec *r) {
    memset(r, 0, sizeof *r);
    for (int i = 0; i < 16; ++i) {
        r->memory[i] = n->memory[i];
        r->dir_bv[i] = n->directory[i].bitVector;
        r->dir_state[i] = (uint8_t)n->directory[i].state;
    }
    for (int i = 0; i < 4; ++i) {
        r->cache_addr[i] = n->cache[i].address;
        r->cache_value[i] = n->cache[i].value;
        r->cache_state[i] = (uint8_t)n->cache[i].state;
    }
    r->pending = n->pendingWriteValue;
    r->flags = (uint8_t)((waiting ? 1 : 0) | (done ? 2 : 0));
    r->issued = (uint16_t)issued;
}

/* main :137-146 locals, then the lock-step schedule in place of :153-699 */
static void reset_ctx(int t) {
    memset(&C[t], 0, sizeof C[t]);
    C[t].instructionIdx = -1;
    C[t].instructions_done = 0;
    C[t].node.waitingForReply = 0;
    C[t].node.pendingWriteValue = 0;
    C[t].node.outstandingMsgs = 0;
}

/* seeded schedule exploration (dsm_common.h dsm_sched_act); lock-step by default */
static uint64_t g_sched_seed, g_sys;
static uint32_t g_sched_thresh = DSM_SCHED_LOCKSTEP;
/* round limit: DSM_ROUND_LIMIT, or DSM_REF_ROUND_LIMIT from the environment (tests) */
static uint32_t g_round_limit = DSM_ROUND_LIMIT;
/* inbox limit: MSG_BUFFER_SIZE (:12), or DSM_REF_INBOX_LIMIT (tests; <= MSG_BUFFER_SIZE) */
static int g_inbox_limit = MSG_BUFFER_SIZE;

/* handled messages of the last run_system by transactionType (:20-34), for the aggregates'
 * msgs_by_type */
static uint64_t g_sys_types[13];

static void run_system(dsm_res *res, dsm_rec *dump, dsm_rec *fin) {
    uint32_t rounds = 0, msgs = 0, instrs = 0, status = ST_COMPLETED;
    g_assert_failed = 0;
    memset(g_sys_types, 0, sizeof g_sys_types);
    for (uint32_t r = 1;; ++r) {
        int acted = 0;
        nst = 0;
        for (int t = 0; t < NUM_PROCS; ++t) {
            nodeCtx *c = &C[t];
            if (g_sched_thresh < DSM_SCHED_LOCKSTEP) {
                const int avail = c->count > 0 ||
                    (!(c->node.waitingForReply > 0) && !c->instructions_done);
                if (avail && !dsm_sched_act(g_sched_seed, g_sched_thresh, g_sys, r, t)) {
                    acted = 1;
                    continue;
                }
            }
            if (c->count > 0) {
                message m = c->ring[c->head];
                c->head = (c->head + 1) % MSG_BUFFER_SIZE;
                c->count--;
                if ((unsigned)m.type < 13u) g_sys_types[m.type]++;
                handle(t, c, m);
                acted = 1; msgs++;
            } else if (c->node.waitingForReply > 0) {
            } else if (!c->instructions_done) {
                int before = c->instructionIdx;
                issue(t, c);
                if (c->instructionIdx != before) instrs++;
                acted = 1;
            }
        }
        if (g_assert_failed) { status = ST_ASSERT_FAILED; rounds = r; break; }
        int ovf = (nst > MAX_STAGED);
        for (int k = 0; k < nst && !ovf; ++k) {
            nodeCtx *d = &C[st_dest[k]];
            if (d->count >= g_inbox_limit) { ovf = 1; break; }
            d->ring[(d->head + d->count) % MSG_BUFFER_SIZE] = st_msg[k];
            d->count++;
        }
        if (ovf) { status = ST_RING_OVERFLOW; rounds = r; break; }
        if (!acted) {
            int all = 1;
            for (int t = 0; t < NUM_PROCS; ++t) all &= C[t].dumped;
            status = all ? ST_COMPLETED : ST_DEADLOCKED;
            break;
        }
        rounds = r;
        if (r >= g_round_limit) { status = ST_ROUND_LIMIT; break; }
    }
    uint32_t mask = 0;
    uint64_t dh = 0, fh = 0;
    for (int t = 0; t < NUM_PROCS; ++t) {
        memset(&dump[t], 0, sizeof dump[t]);
        if (C[t].dumped) {
            mask |= 1u << t;
            to_rec(&C[t].dumpSnap, C[t].dumpSnap.waitingForReply, 1,
                   C[t].instructionIdx + 1, &dump[t]);
            dh += dsm_hash_rec(t, &dump[t], DSM_DUMP_WORDS);
        }
        to_rec(&C[t].node, C[t].node.waitingForReply, C[t].instructions_done,
               C[t].instructionIdx + 1, &fin[t]);
        fh += dsm_hash_rec(t, &fin[t], DSM_FINAL_WORDS);
    }
    res->status = status | (mask << 8);
    res->rounds = rounds; res->msgs = msgs; res->instrs = instrs;
    res->dump_hash = dh; res->final_hash = fh;
}

static void write_sys(FILE *f, const dsm_res *res, const dsm_rec *dump, const dsm_rec *fin) {
    fwrite(res, sizeof *res, 1, f);
    fwrite(dump, sizeof(dsm_rec), NUM_PROCS, f);
    fwrite(fin, sizeof(dsm_rec), NUM_PROCS, f);
}

/* full-size golden aggregates (gen_fixtures.py aggregates; bench.py checks the GPU's against
 * them): sums over systems, status counts, max rounds, and a per-system result digest
 * (dsm_result_digest, dsm_common.h: position-sensitive, so it pins every system's result,
 * not only the totals) */
typedef struct {
    uint64_t systems, msgs, instrs, rounds, max_rounds, status[5], dh, fh, digest, ns;
    uint64_t types[13];
} agg_t;

static void agg_add(agg_t *a, uint64_t idx, const dsm_res *r) {
    for (int k = 0; k < 13; ++k) a->types[k] += g_sys_types[k];
    a->systems++;
    a->msgs += r->msgs; a->instrs += r->instrs; a->rounds += r->rounds;
    if (r->rounds > a->max_rounds) a->max_rounds = r->rounds;
    if ((r->status & 0xFFu) < 5u) a->status[r->status & 0xFFu]++;
    a->dh += r->dump_hash; a->fh += r->final_hash;
    a->digest += dsm_result_digest(idx, r->status, r->rounds, r->msgs, r->instrs,
                                   r->dump_hash, r->final_hash);
}

static void agg_merge(agg_t *a, const agg_t *b) {
    a->systems += b->systems; a->msgs += b->msgs; a->instrs += b->instrs; a->rounds += b->rounds;
    if (b->max_rounds > a->max_rounds) a->max_rounds = b->max_rounds;
    for (int i = 0; i < 5; ++i) a->status[i] += b->status[i];
    a->dh += b->dh; a->fh += b->fh; a->digest += b->digest;
    for (int k = 0; k < 13; ++k) a->types[k] += b->types[k];
}

int main(int argc, char **argv) {
    dsm_res res;
    dsm_rec dump[NUM_PROCS], fin[NUM_PROCS];
    {
        const char *e = getenv("DSM_REF_ROUND_LIMIT");
        if (e && *e && strtoul(e, 0, 0) > 0) g_round_limit = (uint32_t)strtoul(e, 0, 0);
        e = getenv("DSM_REF_INBOX_LIMIT");
        if (e && *e && atoi(e) > 0 && atoi(e) <= MSG_BUFFER_SIZE) g_inbox_limit = atoi(e);
    }
    if (argc == 8 && !strcmp(argv[1], "tests")) {
        /* n schedule-exploration variants (system ids first .. first+n-1) of one test */
        g_sched_seed = strtoull(argv[4], 0, 0);
        g_sched_thresh = (uint32_t)strtoul(argv[5], 0, 0);
        const uint64_t first = strtoull(argv[6], 0, 0), n = strtoull(argv[7], 0, 0);
        FILE *f = fopen(argv[3], "wb");
        if (!f) { perror("open out"); return 1; }
        for (uint64_t k = 0; k < n; ++k) {
            g_sys = first + k;
            for (int t = 0; t < NUM_PROCS; ++t) {
                reset_ctx(t);
                initializeProcessor(t, &C[t].node, argv[2]);
            }
            run_system(&res, dump, fin);
            write_sys(f, &res, dump, fin);
        }
        fclose(f);
        return 0;
    }
    if (argc == 4 && !strcmp(argv[1], "tests")) {
        FILE *f = fopen(argv[3], "wb");
        if (!f) { perror("open out"); return 1; }
        g_write_files = 1;
        for (int t = 0; t < NUM_PROCS; ++t) {
            reset_ctx(t);
            initializeProcessor(t, &C[t].node, argv[2]);
        }
        fflush(stdout);
        run_system(&res, dump, fin);
        write_sys(f, &res, dump, fin);
        fclose(f);
        return 0;
    }
    if (argc == 8 && !strcmp(argv[1], "gen")) {
        int dist = atoi(argv[2]);
        uint64_t seed = strtoull(argv[3], 0, 0);
        int n_instr = atoi(argv[4]);
        uint64_t first = strtoull(argv[5], 0, 0), n = strtoull(argv[6], 0, 0);
        if (n_instr > MAX_INSTR_NUM) { fprintf(stderr, "n_instr > MAX_INSTR_NUM\n"); return 1; }
        FILE *f = fopen(argv[7], "wb");
        if (!f) { perror("open out"); return 1; }
        /* initializeProcessor reads tests/<dir>/core_n.txt: give it empty files in a
         * scratch CWD, then install the generated instructions (:802-818 layout). */
        char tmpl[] = "/tmp/reflsXXXXXX";
        if (!mkdtemp(tmpl) || chdir(tmpl)) { perror("scratch"); return 1; }
        mkdir("tests", 0700); mkdir("tests/empty", 0700);
        for (int t = 0; t < NUM_PROCS; ++t) {
            char p[64]; snprintf(p, sizeof p, "tests/empty/core_%d.txt", t);
            FILE *e = fopen(p, "w"); if (e) fclose(e);
        }
        if (!freopen("/dev/null", "w", stdout)) return 1;
        for (uint64_t s = 0; s < n; ++s) {
            for (int t = 0; t < NUM_PROCS; ++t) {
                reset_ctx(t);
                initializeProcessor(t, &C[t].node, "empty");
                for (int i = 0; i < n_instr; ++i) {
                    uint16_t w = dsm_gen_instr(seed, dist, NUM_PROCS, first + s, t, (uint32_t)i);
                    C[t].node.instructions[i].type = (w >> 15) ? 'W' : 'R';
                    C[t].node.instructions[i].address = (byte)((w >> 8) & 0x7F);
                    C[t].node.instructions[i].value = (byte)(w & 0xFF);
                }
                C[t].node.instructionCount = n_instr;
            }
            run_system(&res, dump, fin);
            write_sys(f, &res, dump, fin);
        }
        fclose(f);
        for (int t = 0; t < NUM_PROCS; ++t) {
            char p[64]; snprintf(p, sizeof p, "tests/empty/core_%d.txt", t); unlink(p);
        }
        rmdir("tests/empty"); rmdir("tests"); if (chdir("/")) {} rmdir(tmpl);
        return 0;
    }
    if (argc == 8 && (!strcmp(argv[1], "bench") || !strcmp(argv[1], "agg"))) {
        /* bench: CPU baseline -- the reference's own handler text under the lock-step
         * schedule over systems first .. first+n-1 of the generator, in nproc forked
         * processes (one slice each).  Only run_system is timed (CLOCK_MONOTONIC around each
         * call): trace generation and initializeProcessor's file reads stay outside, as the
         * GPU's timed region starts with the traces resident in HBM.
         * agg: the same run, reported as the full-size golden aggregates (agg_add): counters,
         * status counts, hash sums and a per-system result digest.  Prints one JSON line. */
        const int is_agg = !strcmp(argv[1], "agg");
        int dist = atoi(argv[2]);
        uint64_t seed = strtoull(argv[3], 0, 0);
        int n_instr = atoi(argv[4]);
        uint64_t first = strtoull(argv[5], 0, 0), n = strtoull(argv[6], 0, 0);
        int nproc = atoi(argv[7]);
        if (n_instr > MAX_INSTR_NUM || nproc < 1 || nproc > 256) { fprintf(stderr, "bad args\n"); return 1; }
        int fds[256][2];
        for (int p = 0; p < nproc; ++p) {
            if (pipe(fds[p])) { perror("pipe"); return 1; }
            pid_t pid = fork();
            if (pid < 0) { perror("fork"); return 1; }
            if (pid == 0) {
                close(fds[p][0]);
                const uint64_t lo = first + n * (uint64_t)p / (uint64_t)nproc;
                const uint64_t hi = first + n * (uint64_t)(p + 1) / (uint64_t)nproc;
                char tmpl[] = "/tmp/refbenchXXXXXX";
                if (!mkdtemp(tmpl) || chdir(tmpl)) _exit(1);
                mkdir("tests", 0700); mkdir("tests/empty", 0700);
                for (int t = 0; t < NUM_PROCS; ++t) {
                    char q[64]; snprintf(q, sizeof q, "tests/empty/core_%d.txt", t);
                    FILE *e = fopen(q, "w"); if (e) fclose(e);
                }
                if (!freopen("/dev/null", "w", stdout)) _exit(1);
                agg_t a;
                memset(&a, 0, sizeof a);
                for (uint64_t sy = lo; sy < hi; ++sy) {
                    for (int t = 0; t < NUM_PROCS; ++t) {
                        reset_ctx(t);
                        initializeProcessor(t, &C[t].node, "empty");
                        for (int i = 0; i < n_instr; ++i) {
                            uint16_t w = dsm_gen_instr(seed, dist, NUM_PROCS, sy, t, (uint32_t)i);
                            C[t].node.instructions[i].type = (w >> 15) ? 'W' : 'R';
                            C[t].node.instructions[i].address = (byte)((w >> 8) & 0x7F);
                            C[t].node.instructions[i].value = (byte)(w & 0xFF);
                        }
                        C[t].node.instructionCount = n_instr;
                    }
                    struct timespec ta, tb;
                    clock_gettime(CLOCK_MONOTONIC, &ta);
                    run_system(&res, dump, fin);
                    clock_gettime(CLOCK_MONOTONIC, &tb);
                    a.ns += (uint64_t)(tb.tv_sec - ta.tv_sec) * 1000000000ull + (uint64_t)(tb.tv_nsec - ta.tv_nsec);
                    agg_add(&a, sy, &res);   /* absolute system id: shards merge */
                }
                for (int t = 0; t < NUM_PROCS; ++t) {
                    char q[64]; snprintf(q, sizeof q, "tests/empty/core_%d.txt", t); unlink(q);
                }
                rmdir("tests/empty"); rmdir("tests"); if (chdir("/")) {} rmdir(tmpl);
                if (write(fds[p][1], &a, sizeof a) != (ssize_t)sizeof a) _exit(1);
                _exit(0);
            }
            close(fds[p][1]);
        }
        agg_t tot;
        memset(&tot, 0, sizeof tot);
        uint64_t ns_max = 0, ns_sum = 0;
        int ok = 1;
        for (int p = 0; p < nproc; ++p) {
            agg_t v;
            if (read(fds[p][0], &v, sizeof v) != (ssize_t)sizeof v) ok = 0;
            else { agg_merge(&tot, &v); ns_sum += v.ns; if (v.ns > ns_max) ns_max = v.ns; }
            close(fds[p][0]);
        }
        int stt;
        while (wait(&stt) > 0) {}
        if (!ok) { fprintf(stderr, "bench: a worker failed\n"); return 1; }
        if (!is_agg) {
            printf("{\"msgs\": %llu, \"instrs\": %llu, \"systems\": %llu, \"nproc\": %d, "
                   "\"sim_ns_max\": %llu, \"sim_ns_sum\": %llu}\n",
                   (unsigned long long)tot.msgs, (unsigned long long)tot.instrs, (unsigned long long)n, nproc,
                   (unsigned long long)ns_max, (unsigned long long)ns_sum);
        } else {
            printf("{\"systems\": %llu, \"msgs\": %llu, \"instrs\": %llu, \"rounds\": %llu, "
                   "\"max_rounds\": %llu, \"status\": [%llu, %llu, %llu, %llu, %llu], "
                   "\"sum_dump_hash\": \"0x%016llx\", \"sum_final_hash\": \"0x%016llx\", "
                   "\"result_digest\": \"0x%016llx\", \"msgs_by_type\": [",
                   (unsigned long long)tot.systems, (unsigned long long)tot.msgs,
                   (unsigned long long)tot.instrs, (unsigned long long)tot.rounds,
                   (unsigned long long)tot.max_rounds,
                   (unsigned long long)tot.status[0], (unsigned long long)tot.status[1],
                   (unsigned long long)tot.status[2], (unsigned long long)tot.status[3],
                   (unsigned long long)tot.status[4], (unsigned long long)tot.dh,
                   (unsigned long long)tot.fh, (unsigned long long)tot.digest);
            for (int k = 0; k < 13; ++k)
                printf("%s%llu", k ? ", " : "", (unsigned long long)tot.types[k]);
            printf("]}\n");
        }
        return 0;
    }
    if (argc == 4 && !strcmp(argv[1], "fmt")) {
        /* printProcessorState (:824-876) of each 64-byte record of argv[2]; record k is node
         * k % NUM_PROCS.  The reference writes core_<id>_output.txt into the CWD: run in a
         * scratch directory and append each file (u32 length + bytes) to argv[3]. */
        FILE *in = fopen(argv[2], "rb"), *out = fopen(argv[3], "wb");
        if (!in || !out) { perror("open"); return 1; }
        char tmpl[] = "/tmp/reffmtXXXXXX";
        if (!mkdtemp(tmpl) || chdir(tmpl)) { perror("scratch"); return 1; }
        dsm_rec r;
        static char buf[8192];
        for (uint64_t k = 0; fread(&r, sizeof r, 1, in) == 1; ++k) {
            processorNode nd;
            memset(&nd, 0, sizeof nd);
            for (int i = 0; i < MEM_SIZE; ++i) {
                nd.memory[i] = r.memory[i];
                nd.directory[i].bitVector = r.dir_bv[i];
                nd.directory[i].state = (directoryEntryState)r.dir_state[i];
            }
            for (int i = 0; i < CACHE_SIZE; ++i) {
                nd.cache[i].address = r.cache_addr[i];
                nd.cache[i].value = r.cache_value[i];
                nd.cache[i].state = (cacheLineState)r.cache_state[i];
            }
            const int id = (int)(k % NUM_PROCS);
            printProcessorState(id, nd);
            char p[64];
            snprintf(p, sizeof p, "core_%d_output.txt", id);
            FILE *f = fopen(p, "rb");
            if (!f) { perror("dump"); return 1; }
            uint32_t n = (uint32_t)fread(buf, 1, sizeof buf, f);
            fclose(f);
            unlink(p);
            fwrite(&n, sizeof n, 1, out);
            fwrite(buf, 1, n, out);
        }
        fclose(in);
        fclose(out);
        if (chdir("/")) {}
        rmdir(tmpl);
        return 0;
    }
    fprintf(stderr, "usage: %s tests <name> <out.bin> | gen <dist> <seed> <n_instr> <first> <n> <out.bin> | fmt <recs.bin> <out.bin>\n", argv[0]);
    return 2;
}
