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
