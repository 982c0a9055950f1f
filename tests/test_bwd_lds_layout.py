"""The backward blend's matrix-core A operand in LDS (csrc/gsr_render.hip BwdLDS::uw, gsr_uw_pg): each replay step
writes u / w of one candidate row for the 64 pixels (ds_write_b32), each MFMA lane reads its row's 16 pixels of
one k-group as four 16-byte chunks (ds_read_b128).  Checked exhaustively against the bank model of
MI355X_MICROARCH.md §LDS: the writes conflict-free in each 32-lane half (bank = dword mod 32), the reads
conflict-free in each of the four 16-lane groups of ds_read_b128 (bank = dword mod 64), every (row, pixel) in its
own dword inside the array, and the reader's chunk k holding exactly the writer's pixels 16 g + 4 k .. + 3."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "threestudio-3dgs_amd", "csrc", "gsr_render.hip")


def pg(g):
    """gsr_uw_pg: offset of 16-pixel group g."""
    return 256 * (g >> 1) + (528 if g & 1 else 0)


def write_addr(r, p):
    return 16 * r + pg(p >> 4) + 4 * (((p >> 2) & 3) ^ ((r >> 2) & 3)) + (p & 3)


def read_addr(lane, k):
    return 16 * (lane & 15) + pg(lane >> 4) + 4 * (k ^ ((lane >> 2) & 3))


def test_source_matches_restatement():
    src = open(SRC).read()
    assert re.search(r"int gsr_uw_pg\(int g\) \{ return 256 \* \(g >> 1\) \+ \(\(g & 1\) \? 528 : 0\); \}", src)
    m = re.search(r"float uw\[4\]\[([^\]]+)\];", src)
    assert m is not None
    size = eval(m.group(1))  # noqa: S307 (a constant expression of the source)
    cells = {write_addr(r, p) for r in range(16) for p in range(64)}
    assert len(cells) == 16 * 64 and max(cells) < size


def test_writes_conflict_free():
    for r in range(16):
        for half in (range(32), range(32, 64)):
            assert len({write_addr(r, p) % 32 for p in half}) == 32, r


def test_reads_conflict_free_and_consistent():
    groups = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
              [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
    groups += [[x + 32 for x in g] for g in groups]
    for k in range(4):
        for g in groups:
            banks = {(read_addr(lane, k) + d) % 64 for lane in g for d in range(4)}
            assert len(banks) == 64, (k, g)
    for lane in range(64):
        for k in range(4):
            for e in range(4):
                # MFMA 16x16x4 k-step i = 4 k + e: lane holds A[row = lane & 15][pixel 16 (lane >> 4) + i]
                assert read_addr(lane, k) + e == write_addr(lane & 15, 16 * (lane >> 4) + 4 * k + e)
