"""GPU tests of the batched grid (dcor_grid_launch / dcor_grid_run_multi; replaces the
expand.grid + mclapply blocks of vert-cor.R:486-554 and ver-cor-subG.R:245-296).

Every replicate of a batched launch must be byte-identical to the per-cell launch of the same
(seed, replicate) (dcor_sim_launch, itself checked against the oracle elsewhere), and every
accumulator byte-identical to dcor_accumulate_launch over that cell's records -- for any mix of
kernel families, any chunking and any sharding over devices."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dc():
    import torch
    assert torch.cuda.is_available()
    import dcor
    return dcor


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.uint64)


def _mixed_cells():
    from dcor.sim import CellSpec
    return [
        CellSpec(n=5000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_001),
        CellSpec(n=1003, rho=-0.3, eps1=1.5, eps2=0.5, seed=1_000_002),                          # m = 11
        CellSpec(n=800, rho=0.2, eps1=1.0, eps2=1.0, normalise=False, seed=1_000_003),             # regen
        CellSpec(n=2500, rho=0.65, eps1=0.5, eps2=0.5, dgp="bernoulli", seed=1_000_004),            # bern_w
        CellSpec(n=20_000, rho=0.4, eps1=1.0, eps2=1.0, dgp="bernoulli", seed=1_000_005),           # bern
        CellSpec(n=3001, rho=0.65, eps1=1.5, eps2=0.5, family="subG", dgp="bounded_factor", seed=1_000_006),
        CellSpec(n=2000, rho=0.3, eps1=1.0, eps2=1.0, family="subG", dgp="mix_gaussian", seed=1_000_007),
        CellSpec(n=1500, rho=0.5, eps1=1.0, eps2=1.0, dgp="mix_gaussian", seed=1_000_008),
        CellSpec(n=1200, rho=0.5, eps1=1.0, eps2=1.0, nsim=2000, seed=1_000_009),                 # VPL 32
        CellSpec(n=900, rho=-0.2, eps1=1.0, eps2=1.0, family="subG", dgp="bounded_factor", seed=1_000_010),  # NaN cell
        CellSpec(n=4000, rho=0.8, eps1=1.0, eps2=1.0, family="subG", dgp="gaussian", seed=1_000_011),
        CellSpec(n=3000, rho=0.1, eps1=0.5, eps2=1.5, family="sign", dgp="bounded_factor", seed=1_000_012),
    ]


def _per_cell(cells, begins, counts):
    from dcor.sim import accum_from_bytes, accumulate, simulate
    recs, accs = [], []
    for c, b, n in zip(cells, begins, counts):
        r = simulate(c, n, b)
        recs.append(r.cpu().numpy())
        accs.extend(bytes(a) for a in accum_from_bytes(accumulate(r, c.rho).cpu().numpy().tobytes()))
    return np.concatenate(recs), accs


def _check_launch(cells, begins, counts):
    from dcor import _lib
    from dcor.sim import grid_launch
    out, acc = grid_launch(cells, begins, counts)
    got = out.cpu().numpy()
    ref, ref_acc = _per_cell(cells, begins, counts)
    assert np.array_equal(_bits(got), _bits(ref))
    raw = acc.cpu().numpy().tobytes()
    sz = len(raw) // (2 * len(cells))
    assert sz == _lib.C.sizeof(_lib.Accum)
    assert [raw[i * sz:(i + 1) * sz] for i in range(2 * len(cells))] == ref_acc


def test_grid_launch_equals_per_cell_launches(dc):
    cells = _mixed_cells()
    counts = [37, 64, 5, 300, 9, 130, 17, 33, 21, 11, 2049, 40]   # 2049: a two-block accumulate
    begins = [0, 7, 1000, 3, 0, 250, 9, 0, 4, 0, 100, 77]
    _check_launch(cells, begins, counts)


def test_grid_launch_chunks_and_streams(dc, variant):
    """A 1 MiB slab budget splits the code items into many chunks over the two streams."""
    variant("DCOR_GRID_SLAB_MB", "1")
    from dcor.sim import CellSpec
    cells = [CellSpec(n=n, rho=0.5, eps1=1.0, eps2=1.0, seed=2_000_000 + n) for n in (3000, 700, 12_345)]
    _check_launch(cells, [0, 5, 11], [300, 129, 260])


def test_grid_launch_empty_cells_and_refusal(dc):
    from dcor import _lib
    from dcor.sim import CellSpec
    cells = [CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, seed=3), CellSpec(n=900, rho=0.1, eps1=1.0, eps2=1.0, seed=4)]
    _check_launch(cells, [0, 0], [0, 12])
    bad = cells + [CellSpec(n=100, rho=0.3, eps1=0.2, eps2=0.2, seed=5)]   # k = floor(100/200) = 0
    from dcor.sim import grid_launch
    with pytest.raises(_lib.DcorError, match="cell 2"):
        grid_launch(bad, 0, 10)


@pytest.mark.parametrize("which", ["vert_cor", "subg"])
def test_reference_grids_B250(dc, which):
    """vert-cor.R's 144-cell and ver-cor-subG.R's 120-cell grids at the reference's B = 250 through
    one dcor_grid_run_multi call: records and accumulators equal the per-cell launches."""
    from dcor.sim import run_grid, subg_grid, vert_cor_grid
    cells = vert_cor_grid() if which == "vert_cor" else subg_grid()
    B = 250
    res = run_grid(cells, B, detail=True, devices=[0])
    got = np.concatenate([r["records"] for r in res])
    ref, ref_acc = _per_cell(cells, [0] * len(cells), [B] * len(cells))
    assert np.array_equal(_bits(got), _bits(ref))
    assert [bytes(a) for r in res for a in r["accum"]] == ref_acc
    cov = [r["summary"]["NI"]["coverage"] for r in res]
    assert 0.85 < float(np.mean(cov)) < 0.99


@pytest.mark.parametrize("devices,B", [([0, 0], 101), ([0, 0, 0], 250)])
def test_grid_sharded_over_devices(dc, devices, B):
    """The same device listed G times: G host threads, each with its own scratch and streams,
    run the replicate ranges [g B / G, (g+1) B / G).  Records equal the unsharded run byte for
    byte; merged accumulators: counts exact, sums within 1e-15 relative."""
    from dcor.sim import run_grid
    cells = _mixed_cells()
    one = run_grid(cells, B, detail=True, devices=[0])
    many = run_grid(cells, B, detail=True, devices=devices)
    for a, b in zip(one, many):
        assert np.array_equal(_bits(a["records"]), _bits(b["records"]))
        for x, y in zip(a["accum"], b["accum"]):
            for f in ("n", "n_cover", "n_cover_na", "n_na_est", "n_na_ci"):
                assert getattr(x, f) == getattr(y, f)
            for f in ("est", "est2", "se2", "len", "lo", "hi"):
                u, v = getattr(x, f)[0] + getattr(x, f)[1], getattr(y, f)[0] + getattr(y, f)[1]
                assert u == v or abs(u - v) <= 1e-15 * max(abs(u), abs(v)) or (np.isnan(u) and np.isnan(v))


def test_two_host_threads_on_one_device(dc):
    """dcor_sim_launch from two host threads at once, each on its own stream: per-thread scratch
    and auxiliary streams keep the one-pass sign pipeline's slabs apart."""
    import torch
    from dcor.sim import CellSpec, simulate
    cells = [CellSpec(n=20_000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=s)
             for s in (1_000_021, 1_000_022)]
    ref = [simulate(c, 1536, 0).cpu().numpy() for c in cells]
    got = [None, None]

    def work(i):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out = torch.empty((1536, 6), dtype=torch.float64, device="cuda")
            for _ in range(3):
                simulate(cells[i], 1536, 0, out=out, stream=s)
            got[i] = out.cpu().numpy()

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for g, r in zip(got, ref):
        assert np.array_equal(_bits(g), _bits(r))


def test_grid_run_multi_persistent_workers_allocate_once(dc):
    """dcor_grid_run_multi keeps one persistent worker per (device, listing): a second call with the
    same device list and grid makes no new device or pinned allocation (dcor_alloc_count), for the
    calling-thread path (one device) and the worker path (device 0 listed twice)."""
    from dcor import _lib
    from dcor.sim import run_grid
    cells = _mixed_cells()
    for devices in ([0], [0, 0]):
        first = run_grid(cells, 101, detail=True, devices=devices)
        n0 = _lib.lib.dcor_alloc_count()
        again = run_grid(cells, 101, detail=True, devices=devices)
        assert _lib.lib.dcor_alloc_count() == n0, devices
        for a, b in zip(first, again):
            assert np.array_equal(_bits(a["records"]), _bits(b["records"]))
            assert [bytes(x) for x in a["accum"]] == [bytes(x) for x in b["accum"]]


def test_grid_memory_bounded_in_B(dc, variant):
    """Device memory does not grow with B: with a 1 MiB record buffer the replicates
    run in many passes of whole accumulate blocks; the accumulators are still byte-identical to
    one dcor_accumulate_launch over each cell's records, the detail records to the per-cell
    launches, and a 4x larger B holds the same device bytes."""
    from dcor import _lib
    from dcor.sim import CellSpec, run_grid
    variant("DCOR_GRID_REC_MB", "1")            # 21,845 records per pass
    variant("DCOR_GRID_CHUNK_ITEMS", "4096")    # and many chunks per pass
    cells = [CellSpec(n=1000, rho=0.3, eps1=1.0, eps2=1.0, family="subG", dgp="bounded_factor", seed=1_000_031),
             CellSpec(n=1200, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_032),
             CellSpec(n=900, rho=0.65, eps1=0.5, eps2=0.5, dgp="bernoulli", seed=1_000_033)]
    B = 30_011      # 15 accumulate blocks per cell, passes split cells
    res = run_grid(cells, B, detail=True, devices=[0])
    ref, ref_acc = _per_cell(cells, [0] * 3, [B] * 3)
    assert np.array_equal(_bits(np.concatenate([r["records"] for r in res])), _bits(ref))
    assert [bytes(a) for r in res for a in r["accum"]] == ref_acc
    run_grid(cells, 20_000, devices=[0])
    held = _lib.lib.dcor_device_bytes()
    res4 = run_grid(cells, 4 * 20_000, devices=[0])          # no detail: accumulators only
    # only the block partials may grow (<= 512 per cell, 2 x 160 B each), never the record buffer
    assert _lib.lib.dcor_device_bytes() - held <= 3 * 512 * 2 * 160
    assert all(r["accum"][0].n == 80_000 for r in res4)


def test_two_host_threads_run_multi_concurrently(dc):
    """dcor_grid_run_multi from two host threads at once, each with two shards on
    device 0 (persistent workers): every thread's accumulators and records equal its serial run."""
    from dcor.sim import CellSpec, run_grid
    grids = [_mixed_cells()[:4],
             [CellSpec(n=4000, rho=0.3, eps1=1.0, eps2=1.0, family="subG", dgp="bounded_factor", seed=1_000_201),
              CellSpec(n=6000, rho=-0.5, eps1=1.5, eps2=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_202)]]
    ref = [run_grid(g, 257, detail=True, devices=[0, 0]) for g in grids]
    got = [None, None]
    err = []

    def work(i):
        try:
            for _ in range(3):
                got[i] = run_grid(grids[i], 257, detail=True, devices=[0, 0])
        except Exception as e:  # noqa: BLE001 -- reported below
            err.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    for g, r in zip(got, ref):
        for a, b in zip(g, r):
            assert np.array_equal(_bits(a["records"]), _bits(b["records"]))
            assert [bytes(x) for x in a["accum"]] == [bytes(x) for x in b["accum"]]
