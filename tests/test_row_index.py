"""Row-group index of sorted loader rows (csrc_host/row_index.h) and the per-rank row selection
on it (csrc_host/shard_rows.cpp, mfa_shard_rows_ix): against numpy on random panels, the order
checks at every thread-chunk boundary, and the index the CSV reader builds while parsing."""
import numpy as np
import pytest

from llm_driven_multi_factor_model_amd.utils import native_io as nio


def _panel(seed, nstk=37, tmax=60, with_ed=True):
    rng = np.random.default_rng(seed)
    cal = np.array(sorted(set(20150105 + rng.choice(3000, 400, replace=False))), dtype=np.int32)
    cal = cal[(cal % 100 >= 1) & (cal % 100 <= 28) & (cal // 100 % 100 >= 1) & (cal // 100 % 100 <= 12)]
    codes, dates, eds = [], [], []
    for k in range(nstk):
        n = int(rng.integers(1, tmax))
        d = np.sort(rng.choice(cal, size=min(n, cal.size), replace=False))
        codes.append(np.full(d.size, b"%06d.SZ" % (k * 7 + 3), dtype="S16"))
        dates.append(d)
        eds.append(np.sort(rng.integers(0, 5, d.size)).astype(np.int32) + 20150000 + 100 * k)
    return np.concatenate(codes), np.concatenate(dates).astype(np.int32), np.concatenate(eds)


@pytest.mark.parametrize("nthreads", [1, 3, 7, 16])
def test_row_index_matches_numpy(nthreads):
    codes, dates, _ = _panel(1)
    ix = nio.row_index(codes, dates, nthreads)
    starts = np.flatnonzero(np.r_[True, codes[1:] != codes[:-1]])
    np.testing.assert_array_equal(ix.seg_first, starts)
    np.testing.assert_array_equal(ix.dates, np.unique(dates))
    np.testing.assert_array_equal(nio.trade_dates(dates, nthreads), np.unique(dates))


@pytest.mark.parametrize("nthreads", [1, 2, 5, 16])
def test_row_index_rejects_every_order_violation(nthreads):
    """A swapped pair of codes or a repeated / descending date anywhere -- inside a thread's
    chunk or on the row right after a chunk boundary -- makes the index None."""
    codes, dates, _ = _panel(2, nstk=12, tmax=30)
    R = codes.size
    cuts = {R * t // nthreads for t in range(1, nthreads)}
    rows = sorted(cuts | {1, R // 2 + 1, R - 1})
    for r in rows:
        if r <= 0 or r >= R:
            continue
        if codes[r] == codes[r - 1]:
            bd = dates.copy()
            bd[r] = bd[r - 1]           # repeated date inside a stock
            assert nio.row_index(codes, bd, nthreads) is None, r
        else:
            bc = codes.copy()
            bc[[r - 1, r]] = bc[[r, r - 1]]   # adjacent stocks out of order
            assert nio.row_index(bc, dates, nthreads) is None, r
    # a stock split in two non-adjacent runs
    bc = codes.copy()
    bc[codes == codes[-1]] = codes[0]    # the last stock's rows re-use the first stock's code
    assert nio.row_index(bc, dates, nthreads) is None


def _ref_select(codes, dates, eds, date_lo, date_hi, halo, nstmt=4):
    starts = np.flatnonzero(np.r_[True, codes[1:] != codes[:-1]])
    ends = np.r_[starts[1:], codes.size]
    out = []
    for k, (a, b) in enumerate(zip(starts, ends)):
        d = dates[a:b]
        klo = a + int(np.searchsorted(d, date_lo))
        khi = a + int(np.searchsorted(d, date_hi))
        if klo >= khi:
            continue
        s = max(a, klo - halo)
        if eds is not None:
            seen, j = [], klo - 1
            while j >= a:
                if not seen or eds[j] != seen[-1]:
                    if len(seen) == nstmt:
                        break
                    seen.append(eds[j])
                j -= 1
            s = min(s, j + 1)
        out.append((s, khi, k))
    return out


@pytest.mark.parametrize("seed,halo,with_ed", [(3, 5, True), (4, 0, False), (5, 40, True)])
def test_shard_rows_ix_matches_reference(seed, halo, with_ed):
    codes, dates, eds = _panel(seed)
    eds = eds if with_ed else None
    ix = nio.row_index(codes, dates)
    dv = ix.dates
    for lo, hi in ((0, dv.size // 3), (dv.size // 3, 2 * dv.size // 3), (2 * dv.size // 3, dv.size)):
        big = np.iinfo(np.int32).max
        dlo = int(dv[lo]) if lo < dv.size else big
        dhi = int(dv[hi]) if hi < dv.size else big
        ranges, sid = nio.shard_rows_ix(ix, dates, eds, dlo, dhi, halo)
        ref = _ref_select(codes, dates, eds, dlo, dhi, halo)
        assert [(int(a), int(b), int(k)) for (a, b), k in zip(ranges, sid)] == ref


def test_csv_reader_builds_the_index_while_parsing(tmp_path):
    codes, dates, _ = _panel(6, nstk=50, tmax=80)
    rng = np.random.default_rng(0)
    close = rng.random(codes.size)
    path = tmp_path / "p.csv"
    with open(path, "w") as f:
        f.write("ts_code,trade_date,close\n")
        for c, d, x in zip(codes, dates, close):
            f.write(f"{c.decode()},{d},{x:.6f}\n")
    types = {"ts_code": 1, "trade_date": 2, "close": 3}
    for nt in (1, 4, 9):
        got = nio.read_columns(str(path), types, nthreads=nt, index=("ts_code", "trade_date"))
        ix = got[nio.ROW_INDEX]
        ref = nio.row_index(got["ts_code"], got["trade_date"])
        np.testing.assert_array_equal(ix.seg_first, ref.seg_first)
        np.testing.assert_array_equal(ix.dates, ref.dates)
        np.testing.assert_array_equal(got["trade_date"], dates)
    # rows out of (code, date) order: columns parsed, no index
    with open(path, "w") as f:
        f.write("ts_code,trade_date,close\n")
        for c, d, x in list(zip(codes, dates, close))[::-1]:
            f.write(f"{c.decode()},{d},{x:.6f}\n")
    got = nio.read_columns(str(path), types, nthreads=4, index=("ts_code", "trade_date"))
    assert nio.ROW_INDEX not in got and got["trade_date"].size == codes.size


def _indexed_vs_key(device, pinned):
    """DeviceFactorEngine built from the reader's row-group index (no code upload, ids from the
    segments, dates by searchsorted) == the key-based build (device unique of the S16 codes and
    dates): same ids, axes, columns and descriptors."""
    import torch
    from llm_driven_multi_factor_model_amd.models import e2e
    from llm_driven_multi_factor_model_amd.models import factor_engine as FE
    prices, index, _ = FE.synthetic_prices(N=40, T=300, seed=2, n_ind=31)
    prices = prices.sort_values(["ts_code", "trade_date"], kind="stable").reset_index(drop=True)
    p, i = e2e._columns_from_frames(prices, index)
    p["trade_date"] = p["trade_date"].astype("int32")
    if "end_date" in p:
        p["end_date"] = p["end_date"].astype("int32")
    ps = e2e.stage_host_columns(p, pinned=pinned)
    assert nio.ROW_INDEX in ps
    a = e2e.DeviceFactorEngine(dict(ps), dict(i), device=device)
    b = e2e.DeviceFactorEngine({k: v for k, v in ps.items() if k != nio.ROW_INDEX}, dict(i),
                               device=device)
    assert torch.equal(a.stock_id, b.stock_id) and torch.equal(a.date_id, b.date_id)
    assert (a.date_ints == b.date_ints).all() and list(a.stock_names) == list(b.stock_names)
    for k in b.cols:
        assert torch.equal(a.cols[k].nan_to_num(7.0), b.cols[k].nan_to_num(7.0)), k
    ra, rb = a.compute(FE.FACTORS_TO_RUN), b.compute(FE.FACTORS_TO_RUN)
    for k in rb:
        assert torch.equal(ra[k].nan_to_num(7.0), rb[k].nan_to_num(7.0)), k


def test_device_engine_indexed_build_equals_key_build():
    _indexed_vs_key("cpu", False)


@pytest.mark.gpu
def test_device_engine_indexed_build_equals_key_build_gpu(cuda):
    _indexed_vs_key(cuda, True)
