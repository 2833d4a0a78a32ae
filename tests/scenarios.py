"""Hand-built systems, one per protocol quirk of the reference.
Expected values were derived by hand from assignment.c under the lock-step schedule; the
derivation is written next to each scenario.  Records are dsm_node_state (64 bytes).
"""
import numpy as np

M, E, S, I = 0, 1, 2, 3      # cacheLineState :17
EM, DS, DU = 0, 1, 2         # directoryEntryState :18
COMPLETED, DEADLOCKED = 0, 1


def pk(op, addr, val=0):
    return ((1 if op == "WR" else 0) << 15) | (addr << 8) | (val if op == "WR" else 0)


def build(np_, progs, stride=32):
    tr = np.zeros((1, np_, stride), dtype=np.uint16)
    cn = np.zeros((1, np_), dtype=np.uint32)
    for n, prog in enumerate(progs):
        for i, ins in enumerate(prog):
            tr[0, n, i] = pk(*ins)
        cn[0, n] = len(prog)
    return tr, cn


def line(rec, i):
    return int(rec[48 + i]), int(rec[52 + i]), int(rec[56 + i])


def mem(rec, i):
    return int(rec[i])


def dirent(rec, i):
    return int(rec[32 + i]), int(rec[16 + i])   # (state, bitVector)


SCENARIOS = {}


def scenario(fn):
    SCENARIOS[fn.__name__] = fn
    return fn


@scenario
def write_miss_writes_home_memory():
    """WR 0x15 100 by node 0.  R1 WRITE_REQUEST->1 (nodes 1-3 dump); R2 home writes memory
    first (:379), U->EM{0}, REPLY_WR; R3 node 0 installs M 100; R4 node 0 dumps; R5 idle."""
    tr, cn = build(4, [[("WR", 0x15, 100)], [], [], []])

    def check(res, dump, fin):
        assert int(res["status"]) == COMPLETED | (0xF << 8)
        assert (int(res["rounds"]), int(res["msgs"]), int(res["instrs"])) == (4, 2, 1)
        assert mem(fin[1], 5) == 100
        assert dirent(fin[1], 5) == (EM, 0x01)
        assert line(fin[0], 1) == (0x15, 100, M)
        assert mem(dump[1], 5) == 25            # node 1 dumped in round 1 (no instructions)
    return tr, cn, check


@scenario
def flush_invack_loses_the_pending_write():
    """Nodes 0 and 2 both write 0x15 in round 1.  Home handles node 0 first (U->EM{0}),
    then node 2 (memory=7 at :379, EM owner 0 -> WRITEBACK_INV r2=2, bv={2}).  Node 0 flushes
    M 100 with FLUSH_INVACK to home and node 2; node 2 installs the FLUSHED value 100 as M
    (:491-493): its own write of 7 is lost; home memory ends at 100."""
    tr, cn = build(4, [[("WR", 0x15, 100)], [], [("WR", 0x15, 7)], []])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF == COMPLETED
        assert line(fin[2], 1) == (0x15, 100, M)
        assert int(fin[2][60]) == 7              # pendingWriteValue still 7
        assert line(fin[0], 1) == (0x15, 100, I)
        assert mem(fin[1], 5) == 100
        assert dirent(fin[1], 5) == (EM, 0x04)
    return tr, cn, check


@scenario
def ignored_writeback_int_deadlocks_requester():
    """Node 2 reads 0x15 (E), then reads 0x19 (same cache index) and evicts it.  Node 0's
    READ_REQUEST for 0x15 reaches home just before node 2's EVICT_SHARED (sender order), so
    home forwards WRITEBACK_INT to node 2, whose line now holds 0x19: ignored (:265-270).
    Home then handles the eviction: S{0} -> EM and notifies node 0 (:507-515), which has the
    line INVALID, so nothing changes.  Node 0 waits forever: DEADLOCKED, nodes 1-3 dumped."""
    tr, cn = build(4, [[("RD", 0x01), ("RD", 0x15)], [], [("RD", 0x15), ("RD", 0x19)], []])

    def check(res, dump, fin):
        assert int(res["status"]) == DEADLOCKED | (0b1110 << 8)
        assert int(fin[0][61]) & 1 == 1          # node 0 still waitingForReply
        assert line(fin[0], 1) == (0x15, 0, I)
        assert dirent(fin[1], 5) == (EM, 0x01)
        assert line(fin[2], 1) == (0x19, 29, E)
    return tr, cn, check


@scenario
def reply_id_invalidates_sharers():
    """Nodes 0 and 2 read 0x15 (node 0 E, then WRITEBACK_INT/FLUSH makes both S, memory 25).
    Node 3 (after three local actions) writes 0x15: home is S, sends REPLY_ID{0,2} and goes
    EM{3}; node 3 installs M 77 and sends INV to 0 and 2 (:350-362), which invalidate."""
    tr, cn = build(4, [[("RD", 0x15)], [], [("RD", 0x15)],
                       [("RD", 0x30), ("WR", 0x30, 5), ("WR", 0x15, 77)]])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF == COMPLETED
        assert line(dump[0], 1) == (0x15, 25, S)
        assert line(fin[0], 1) == (0x15, 25, I)
        assert line(fin[2], 1) == (0x15, 25, I)
        assert line(fin[3], 1) == (0x15, 77, M)
        assert line(fin[3], 0) == (0x30, 5, M)
        assert mem(fin[1], 5) == 77
        assert dirent(fin[1], 5) == (EM, 0x08)
    return tr, cn, check


@scenario
def home_self_notify_leaves_cache_shared():
    """Home node 1 and node 0 share 0x15.  Node 0 evicts it: home S{0,1} -> EM and notifies
    the remaining sharer, itself (:509-515).  The self-message clears home's own bit and the
    entry goes U/0 (:501-506) while home's cache line stays SHARED."""
    tr, cn = build(4, [[("RD", 0x15), ("RD", 0x19)], [("RD", 0x15)], [], []])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF == COMPLETED
        assert dirent(fin[1], 5) == (DU, 0x00)
        assert line(fin[1], 1) == (0x15, 25, S)
        assert dirent(fin[1], 9) == (EM, 0x01)
        assert line(fin[0], 1) == (0x19, 29, E)
    return tr, cn, check


@scenario
def evict_modified_writes_back():
    """Node 0 writes 0x15 (M 100), write-hits it (M 101, no message), then reads 0x19 (same
    index): EVICT_MODIFIED(101) to home, which stores 101 and goes U/0 (:541-548)."""
    tr, cn = build(4, [[("WR", 0x15, 100), ("WR", 0x15, 101), ("RD", 0x19)], [], [], []])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF == COMPLETED
        assert mem(fin[1], 5) == 101
        assert dirent(fin[1], 5) == (DU, 0x00)
        assert dirent(fin[1], 9) == (EM, 0x01)
        assert line(fin[0], 1) == (0x19, 29, E)
    return tr, cn, check


@scenario
def upgrade_on_shared_write_hit():
    """Nodes 0 and 2 end up sharing 0x15 (memory 25); node 0 reads two of its own blocks on
    other cache indices (0x02, 0x03) meanwhile.  Node 0 then write-hits its SHARED line:
    M immediately with value 9 (:646-659), UPGRADE to home; home S -> REPLY_ID{2}, EM{0};
    node 0 sends INV to node 2."""
    tr, cn = build(4, [[("RD", 0x15), ("RD", 0x02), ("RD", 0x03), ("WR", 0x15, 9)], [],
                       [("RD", 0x15)], []])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF == COMPLETED
        assert line(fin[0], 1) == (0x15, 9, M)
        assert line(fin[2], 1) == (0x15, 25, I)
        assert dirent(fin[1], 5) == (EM, 0x01)
        assert res["msgs"] > 0
    return tr, cn, check


@scenario
def eight_nodes_all_read_one_block():
    """All 8 nodes read 0x35 in round 1: the home serialises them in sender order; the first
    reader gets E, every later one forces WRITEBACK_INT/FLUSH chains.  Checks NP=8 masks."""
    tr, cn = build(8, [[("RD", 0x35)] for _ in range(8)])

    def check(res, dump, fin):
        assert int(res["status"]) & 0xFF in (COMPLETED, DEADLOCKED)
        assert dirent(fin[3], 5)[0] in (EM, DS)
        assert int(res["msgs"]) >= 8
    return tr, cn, check


# ---- rows found by tools/find_scenarios.c (oracle branch probes, shrunk), derived by hand --

@scenario
def read_request_em_owner_is_requester():
    """READ_REQUEST at a home whose EM owner IS the requester (:215-221): REPLY_RD exclusive,
    no WRITEBACK_INT, no directory change.  Home 2 serves 0x21.  R2: node 1 reads (U ->
    EM{1}).  R5: node 0's WRITE_REQUEST(20): EM owner 1 -> WRITEBACK_INV(r2=0), bv {0}.  R6:
    node 1 flushes FLUSH_INVACK(41); home 2's own READ_REQUEST meets EM{0} -> WRITEBACK_INT(r2=2)
    to node 0, S{0,2}.  R7: node 0 installs the flushed 41 as M (its 20 is lost); node 3's
    WRITE_REQUEST(121) meets S{0,2} -> REPLY_ID{0,2}, EM{3}.  R8: the home part of node 1's
    FLUSH_INVACK arrives late and sets EM{r2 = 0} over EM{3} (:478-480); node 0 flushes to the
    home (S); node 3 installs 121 as M and invalidates 0 and 2.  R10: node 0 reads 0x21 again:
    the home is EM{0} with owner == requester, so it answers REPLY_RD(41, exclusive) at R11.
    Node 0 ends EXCLUSIVE while node 3 holds the line MODIFIED."""
    tr, cn = build(4, [[("WR", 0x15, 128), ("WR", 0x21, 20), ("RD", 0x21)], [("RD", 0x21)],
                       [("RD", 0x01), ("RD", 0x21)], [("WR", 0x35, 248), ("WR", 0x21, 121)]])

    def check(res, dump, fin):
        assert int(res["status"]) == COMPLETED | (0xF << 8)
        assert (int(res["rounds"]), int(res["msgs"]), int(res["instrs"])) == (13, 24, 8)
        assert dirent(fin[2], 1) == (EM, 0x01)
        assert mem(fin[2], 1) == 41
        assert line(fin[0], 1) == (0x21, 41, E)
        assert line(fin[3], 1) == (0x21, 121, M)
        assert int(fin[0][60]) == 20               # node 0's pending write, lost
    return tr, cn, check


@scenario
def write_request_em_owner_is_requester():
    """WRITE_REQUEST at a home whose EM owner IS the requester (:410-418): memory takes the
    value first (:379), REPLY_WR, no WRITEBACK_INV, bv unchanged.  Home 1 serves 0x11.  R10:
    the home part of a FLUSH_INVACK with r2 = 3 sets EM{3}.  R12: node 3 write-misses 0x11
    (its line was invalidated) -> WRITE_REQUEST(89); R13: EM owner 3 == requester: memory =
    89, REPLY_WR; R14: node 3 installs 89 as M.  Node 0 also holds 0x11 MODIFIED (155, from a
    REPLY_ID at R10)."""
    tr, cn = build(4, [[("WR", 0x15, 192), ("RD", 0x35), ("WR", 0x11, 155)], [("WR", 0x11, 120)],
                       [("RD", 0x31), ("RD", 0x11)], [("WR", 0x11, 51), ("WR", 0x11, 89)]])

    def check(res, dump, fin):
        assert int(res["status"]) == COMPLETED | (0xF << 8)
        assert (int(res["rounds"]), int(res["msgs"]), int(res["instrs"])) == (15, 25, 8)
        assert mem(fin[1], 1) == 89
        assert dirent(fin[1], 1) == (EM, 0x08)
        assert line(fin[3], 1) == (0x11, 89, M)
        assert line(fin[0], 1) == (0x11, 155, M)
    return tr, cn, check


@scenario
def ignored_writeback_inv_deadlocks_requester():
    """WRITEBACK_INV at a node whose line no longer holds the block (:467-472): ignored, no
    FLUSH_INVACK, so the requester waits forever.  R8: node 0 write-misses 0x19 (its line was
    flushed-invalidated at R7) -> WRITE_REQUEST(6).  R9: home 1 writes 6, EM owner 3 ->
    WRITEBACK_INV(r2=0) to node 3, bv {0}; the same round node 3 evicts 0x19 (M, 29) to take
    0x01.  R10: node 3's line holds 0x01: the WRITEBACK_INV is ignored; home 1 stores the
    evicted 29 over the 6 (EVICT_MODIFIED, :543) and keeps EM{0} (sender 3 not in bv).
    Node 0 deadlocks; nodes 1-3 dump."""
    tr, cn = build(4, [[("WR", 0x25, 199), ("RD", 0x19), ("WR", 0x19, 6)], [], [],
                       [("RD", 0x01), ("WR", 0x19, 48), ("WR", 0x01, 2)]])

    def check(res, dump, fin):
        assert int(res["status"]) == DEADLOCKED | (0b1110 << 8)
        assert (int(res["rounds"]), int(res["msgs"]), int(res["instrs"])) == (12, 17, 6)
        assert int(fin[0][61]) & 1 == 1           # node 0 still waitingForReply
        assert line(fin[0], 1) == (0x19, 0, I)
        assert mem(fin[1], 9) == 29
        assert dirent(fin[1], 9) == (EM, 0x01)
        assert line(fin[3], 1) == (0x01, 2, M)
        assert mem(fin[0], 1) == 2 and dirent(fin[0], 1) == (EM, 0x08)
    return tr, cn, check


@scenario
def write_hit_on_exclusive_is_local():
    """Write hit on an EXCLUSIVE line (:640-645): value and state M locally, no message.
    Node 1 reads its own block 0x19 (R1 READ_REQUEST to itself, R2 U -> EM{1}, R3 installs
    29 EXCLUSIVE), then writes 120 at R4: MODIFIED 120, memory keeps 29; R5 dump."""
    tr, cn = build(4, [[], [("RD", 0x19), ("WR", 0x19, 120)], [], []])

    def check(res, dump, fin):
        assert int(res["status"]) == COMPLETED | (0xF << 8)
        assert (int(res["rounds"]), int(res["msgs"]), int(res["instrs"])) == (5, 2, 2)
        assert line(fin[1], 1) == (0x19, 120, M)
        assert line(dump[1], 1) == (0x19, 120, M)
        assert int(fin[1][60]) == 120
        assert mem(fin[1], 9) == 29
        assert dirent(fin[1], 9) == (EM, 0x02)
    return tr, cn, check
