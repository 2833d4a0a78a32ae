/*
 * oracle/dsm_common.h -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * Definitions shared by the two CPU checkers under oracle/:
 *   - dsm_oracle.c    : clean-room C restatement of the reference's protocol under the
 *                       lock-step schedule,
 *   - ref_lockstep.c  : driver that runs the reference's OWN handler text
 *                       (/root/reference/assignment.c, extracted at build time) under
 *                       the same schedule; output only into oracle/_ref/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load anything
 * built from this directory.  The product (hp-assignment-2_amd/) has its own independent
 * implementation of the node record, the hash and the generator; the tests pin the two
 * against each other.
 *
 * Everything here is the build's own convention (canonical node record, hash, synthetic
 * trace generator); nothing is taken from the reference except the field meanings cited.
 */
#ifndef DSM_ORACLE_COMMON_H
#define DSM_ORACLE_COMMON_H

#include <stdint.h>
#include <string.h>

/* Canonical 64-byte node record (same layout as dsm_node_state in include/dsm.h).
 * Field meanings follow processorNode (assignment.c:70-81):
 *   memory[16]      <- node.memory            (:72)
 *   dir_bv[16]      <- directory[i].bitVector (:48-51, :73)
 *   dir_state[16]   <- directory[i].state     EM=0,S=1,U=2 (:18)
 *   cache_addr[4]   <- cache[i].address       (:42-46, :71)
 *   cache_value[4]  <- cache[i].value
 *   cache_state[4]  <- cache[i].state         M=0,E=1,S=2,I=3 (:17)
 *   pending         <- node.pendingWriteValue (:77)
 *   flags           bit0 waitingForReply (:78), bit1 instructions_done / dumped (:143)
 *   issued          number of instructions issued (instructionIdx+1, :142, :591)
 */
typedef struct dsm_rec {
    uint8_t memory[16];
    uint8_t dir_bv[16];
    uint8_t dir_state[16];
    uint8_t cache_addr[4];
    uint8_t cache_value[4];
    uint8_t cache_state[4];
    uint8_t pending;
    uint8_t flags;
    uint16_t issued;
} dsm_rec;

/* Per-system result record (same layout as dsm_sys_result in include/dsm.h). */
typedef struct dsm_res {
    uint32_t status;   /* bits 0..7 status code, bits 8..15 mask of nodes that dumped */
    uint32_t rounds;   /* active lock-step rounds (last round in which any node acted) */
    uint32_t msgs;     /* messages handled (the "transactions") */
    uint32_t instrs;   /* instructions issued */
    uint64_t dump_hash;  /* sum over dumped nodes of hash(node, snapshot at dump, words 0..14) */
    uint64_t final_hash; /* sum over nodes of hash(node, final record, words 0..15) */
} dsm_res;

enum { ST_COMPLETED = 0, ST_DEADLOCKED = 1, ST_RING_OVERFLOW = 2, ST_ASSERT_FAILED = 3,
       ST_ROUND_LIMIT = 4 };
enum { DIST_UNIFORM = 0, DIST_HOT = 1, DIST_EVICT = 2 };

#define DSM_NTYPES 13
#define DSM_REF_RING_CAP 256     /* MSG_BUFFER_SIZE, assignment.c:12 */
#define DSM_ROUND_LIMIT (1u << 22)

static inline uint64_t dsm_fmix64(uint64_t z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

/* hash of the first nwords little-endian u32 words of a node record */
static inline uint64_t dsm_hash_rec(int node, const dsm_rec *r, int nwords) {
    uint32_t w[16];
    memcpy(w, r, 64);
    uint64_t h = 0x9E3779B97F4A7C15ULL * (uint64_t)(node + 1);
    for (int i = 0; i < nwords; ++i)
        h = dsm_fmix64(h ^ ((uint64_t)w[i] | ((uint64_t)i << 32)));
    return h;
}
#define DSM_DUMP_WORDS 15
#define DSM_FINAL_WORDS 16

/* per-system result digest (the full-size golden aggregates, tests/golden/aggregates.json):
 * summed mod 2^64 over the systems of a workload, idx = the system's index in it.  Sensitive
 * to every field of every system's result and to its position (bench.py computes it from the
 * GPU's per-system results, tests/test_aggregates.py pins the numpy restatement). */
static inline uint64_t dsm_result_digest(uint64_t idx, uint32_t status, uint32_t rounds,
                                         uint32_t msgs, uint32_t instrs, uint64_t dump_hash,
                                         uint64_t final_hash) {
    uint64_t h = dsm_fmix64(idx * 0x9E3779B97F4A7C15ULL + 1u);
    h = dsm_fmix64(h ^ ((uint64_t)status | ((uint64_t)rounds << 32)));
    h = dsm_fmix64(h ^ ((uint64_t)msgs | ((uint64_t)instrs << 32)));
    h = dsm_fmix64(h ^ dump_hash);
    return dsm_fmix64(h ^ final_hash);
}

/* Counter-based synthetic trace generator.  Instruction idx of node `node`
 * of system `sys` depends only on (seed, dist, np, sys, node, idx): results are independent
 * of how systems are batched or sharded over GPUs.  One splitmix64 output feeds 4
 * consecutive instructions (16 bits each: bit 0 WR, bits 1-8 value, bits 9-15 address
 * selector).  Packed u16: bit 15 = WR, bits 8..14 = address (7 bits), bits 0..7 = value
 * (0 for RD, :810). */
static inline uint64_t dsm_splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint16_t dsm_gen_instr(uint64_t seed, int dist, int np, uint64_t sys, int node,
                                     uint32_t idx) {
    uint64_t key = (sys << 16) | ((uint64_t)node << 12) | (uint64_t)((idx & 0xFFF) >> 2);
    uint64_t r = dsm_splitmix(seed * 0x9E3779B97F4A7C15ULL + key);
    uint32_t h = (uint32_t)(r >> (16 * (idx & 3))) & 0xFFFF;
    uint32_t wr = h & 1;
    uint32_t val = wr ? (h >> 1) & 0xFF : 0;
    uint32_t sel = h >> 9;
    uint32_t addr;
    if (dist == DIST_HOT) addr = (sel & 3) * 0x11;                       /* {0x00,0x11,0x22,0x33} */
    else if (dist == DIST_EVICT) addr = (sel & (uint32_t)(np * 4 - 1)) * 4; /* a%4==0 */
    else addr = sel & (uint32_t)(np * 16 - 1);                           /* uniform 0..np*16-1 */
    return (uint16_t)((wr << 15) | (addr << 8) | val);
}

/* Seeded schedule exploration.  In each round every node whose schedule
 * gives it an action (pop its inbox head / issue / dump, Appendix A) takes it only if
 * dsm_sched_act() says so, otherwise it stalls for that round -- a legal interleaving of the
 * reference's free-running threads.  thresh >= 0x10000 is the plain lock-step schedule.  A
 * round counts (and the system continues) while any node HAS an action, taken or not. */
#define DSM_SCHED_LOCKSTEP 0x10000u
static inline int dsm_sched_act(uint64_t seed, uint32_t thresh, uint64_t sys, uint32_t round,
                                int node) {
    if (thresh >= DSM_SCHED_LOCKSTEP) return 1;
    const uint64_t key = (sys << 26) ^ ((uint64_t)round << 3) ^ (uint64_t)node;
    const uint32_t h = (uint32_t)(dsm_splitmix(seed * 0x9E3779B97F4A7C15ULL + key) >> 48);
    return h < thresh;
}

#endif
