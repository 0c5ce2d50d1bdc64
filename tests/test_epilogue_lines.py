"""CPU check of the whole-line store maps of the persistent GEMM epilogues (csrc/gemm_w4.hip: w4_line_pair,
w4_pair_rows and their use in w4_rows / w4_gbwd_rows).  The register layout gives lane (r = lane & 15,
q = lane >> 4) 8 consecutive columns of row r; two such chunks X, Y of a lane cover, over q, one 128-B line of
its row.  After one exchange with lane ^ 8 (DPP row_ror:8) store 1 must write rows 0-7 and store 2 rows 8-15,
every instruction whole lines, every output chunk exactly once with the right data.  This restates the index
maps and checks those properties for the plain (64- and 128-column waves), GEGLU and GEGLU-backward uses."""
import pytest


def cb_of(q):
    return 16 * (q & 1) + 8 * (q >> 1)


def run_pair(chunk_x, chunk_y):
    """chunk_x / chunk_y: q -> line chunk of X / Y.  Returns the two store instructions as lists of
    (lane, row, chunk, data) where data = (source row, source chunk)."""
    X = {lane: (lane & 15, chunk_x(lane >> 4)) for lane in range(64)}
    Y = {lane: (lane & 15, chunk_y(lane >> 4)) for lane in range(64)}
    sel = {lane: (Y if (lane & 8) == 0 else X)[lane] for lane in range(64)}
    rcv = {lane: sel[lane ^ 8] for lane in range(64)}     # row_ror:8 within each 16-lane row = lane ^ 8
    st1, st2 = [], []
    for lane in range(64):
        lo, r, q = (lane & 8) == 0, lane & 15, lane >> 4
        ch = chunk_x(q) if lo else chunk_y(q)
        d1 = X[lane] if lo else rcv[lane]
        d2 = rcv[lane] if lo else Y[lane]
        row1 = r if lo else r - 8                           # w4_pair_rows: own row or the partner's
        row2 = r + 8 if lo else r
        st1.append((lane, row1, ch, d1))
        st2.append((lane, row2, ch, d2))
    return st1, st2


def check(st1, st2):
    written = {}
    for k, st in enumerate((st1, st2)):
        rows = {row for _, row, _, _ in st}
        assert rows == set(range(8 * k, 8 * k + 8))        # store 1: rows 0-7, store 2: rows 8-15
        for row in rows:                                   # whole 128-B lines: all 8 chunks of every row
            assert sorted(ch for _, r, ch, _ in st if r == row) == list(range(8))
        for _, row, ch, data in st:
            assert (row, ch) not in written
            written[(row, ch)] = data
            assert data == (row, ch)                       # the chunk's own data lands there
    assert len(written) == 16 * 8


def test_plain_line_pairs():
    # plain / GELU (w4_rows): X = column pair 2m (chunk cb / 8 of line m), Y = pair 2m + 1 (chunk 4 + cb / 8)
    check(*run_pair(lambda q: cb_of(q) >> 3, lambda q: 4 + (cb_of(q) >> 3)))


def test_geglu_line_pairs():
    # gate|up (w4, 64 h columns per wave): the same map on g, u and h
    check(*run_pair(lambda q: cb_of(q) >> 3, lambda q: 4 + (cb_of(q) >> 3)))


def test_geglu_bwd_line_pairs():
    # dg | du (w4_gbwd_rows): dh columns 32 pp + cb -> output line pp, dg chunk 4 (cb >> 4) + ((cb >> 3) & 1),
    # du two chunks on
    def dg(q):
        return 4 * (cb_of(q) >> 4) + ((cb_of(q) >> 3) & 1)
    check(*run_pair(dg, lambda q: dg(q) + 2))


@pytest.mark.parametrize("pp", [0, 1, 2, 3])
def test_geglu_bwd_output_columns(pp):
    # the interleaved layout: dh column c -> dg at (c >> 4) * 32 + (c & 15), du 16 on; the line chunks above are
    # those columns relative to 2 col0 + 64 pp
    for q in range(4):
        c = 32 * pp + cb_of(q)
        ch = 4 * (cb_of(q) >> 4) + ((cb_of(q) >> 3) & 1)
        assert 64 * pp + 8 * ch == (c >> 4) * 32 + (c & 15)
        assert 64 * pp + 8 * (ch + 2) == (c >> 4) * 32 + (c & 15) + 16

