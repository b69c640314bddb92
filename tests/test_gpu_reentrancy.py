"""Reentrancy of the C-ABI ("Concurrent calls from Julia threads must be safe").

The reference fits the 32 diodes of an exposure from up to 8 Julia threads
(`Threads.@threads`, /root/reference/src/Modulation.jl:387-433); a Julia caller of the drop-in may
equally call the library from several threads at once (one exposure per thread).  Here 8 host
threads (ctypes releases the GIL for the duration of each call) call gpd_demodulateall,
gpd_demodulateall_c32, gpd_fit_batch and gpd_fit_windows concurrently on distinct exposures,
several rounds each, and every record and every output byte must equal the same call made
serially.  Some calls shard over two devices (option fake_gpus: both shards on the one GPU of
the test box), so the per-device locks, the device arenas, the pinned output staging and the
host copy pool are all crossed by concurrent callers.  No call may take longer than the
deadlock guard.
"""
import threading
import time

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

N = 40_000
ROUNDS = 3
THREADS = 8
DEADLOCK_S = 60.0


def _exposure(gpu, seed):
    """(t, data (N, 40) complex128 column-major) like test_demodulateall_one_exposure_full_size."""
    B = synth.make_batch(N, 32, seed=seed)
    data = np.empty((40, N), dtype=np.complex128)  # column k contiguous: a Julia Matrix
    data[:32] = B["d"]
    fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)])
    for g in range(8):
        cols = np.nonzero(fop == 32 + g)[0]
        data[32 + g] = B["fc"][B["fc_of_pixel"][cols[0]]]
    return B["t"], data.T  # (N, 40) view, column-major


def _states(seed):
    rng = np.random.default_rng(seed)
    st = np.full(N, 2, dtype=np.int8)
    i = N // 10
    while i < N - N // 10:
        hi = int(rng.integers(N // 40, N // 20))
        st[i:i + hi] = 3
        st[i:i + 5] = -1
        lo = int(rng.integers(N // 20, N // 8))
        st[i + hi:i + hi + lo] = 1
        st[i + hi:i + hi + 15] = -1
        i += hi + lo
    return st


def _jobs(gpu):
    """One job per thread: a closure returning the bytes of every record and output."""
    jobs = []
    for j in range(THREADS):
        t, data = _exposure(gpu, 100 + j)
        kind = j % 4
        if kind == 0:  # the drop-in, complex128, faint states on odd exposures
            st = _states(j) if j % 8 == 4 else None

            def run(t=t, data=data, st=st, ng=1 + (j // 4) % 2):
                out, par, lk = gpu.demodulateall(t, data, faintparam=st, n_gpus=ng)
                return [np.asarray(out).tobytes(order="A"), lk.tobytes(),
                        np.array([(p.a, p.b, p.ϕ) for p in par]).tobytes()]
        elif kind == 1:  # the drop-in on Matrix{ComplexF32}
            d32 = np.asfortranarray(data.astype(np.complex64))

            def run(t=t, data=d32, ng=1 + (j // 4) % 2):
                out, par, lk = gpu.demodulateall(t, data, n_gpus=ng)
                assert out.dtype == np.complex64
                return [np.asarray(out).tobytes(order="A"), lk.tobytes()]
        elif kind == 2:  # gpd_fit_batch with the demodulated series, exact on one of them
            cols = np.ascontiguousarray(data.T)
            fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)
            method = "exact" if j == 2 else "auto"

            def run(t=t, cols=cols, fop=fop, method=method, ng=1 + (j // 4) % 2):
                par, out = gpu.fit_batch(t, cols[:32], cols, fop, want_output=True,
                                         method=method, n_gpus=ng)
                return [par.tobytes(), out.tobytes()]
        else:  # gpd_fit_windows, 1-s windows (500 samples at 2 ms)
            cols = np.ascontiguousarray(data.T)
            fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)

            def run(t=t, cols=cols, fop=fop, ng=1 + (j // 4) % 2):
                par, out = gpu.fit_windows(t, cols[:32], cols, fop, 500, want_output=True,
                                           n_gpus=ng)
                return [par.tobytes(), out.tobytes()]
        jobs.append(run)
    return jobs


def test_concurrent_calls_equal_serial_calls(gpu, opts):
    opts("fake_gpus", 1)  # n_gpus = 2 calls: two shards on the one GPU, from two threads each
    jobs = _jobs(gpu)
    for run in jobs:  # warm the device contexts, arenas and staging buffers
        run()
    t0 = time.perf_counter()
    serial = [run() for run in jobs]
    t_serial = time.perf_counter() - t0

    results = [[None] * ROUNDS for _ in jobs]
    errors = []
    start = threading.Barrier(len(jobs))

    def worker(j):
        try:
            start.wait()
            for r in range(ROUNDS):
                results[j][r] = jobs[j]()
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append((j, repr(e)))

    th = [threading.Thread(target=worker, args=(j,), daemon=True) for j in range(len(jobs))]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=max(1.0, DEADLOCK_S - (time.perf_counter() - t0)))
    t_conc = time.perf_counter() - t0
    assert not any(x.is_alive() for x in th), "concurrent calls did not finish (deadlock?)"
    assert not errors, errors
    for j, run in enumerate(jobs):
        for r in range(ROUNDS):
            assert results[j][r] is not None
            for a, b in zip(results[j][r], serial[j]):
                assert a == b, f"job {j} round {r}: concurrent result differs from the serial call"
    calls = len(jobs) * ROUNDS
    print(f"{calls} concurrent calls from {len(jobs)} threads: {t_conc * 1e3:.1f} ms "
          f"({calls / t_conc:.1f} calls/s); serial: {len(jobs)} calls in {t_serial * 1e3:.1f} ms "
          f"({len(jobs) / t_serial:.1f} calls/s) — every result byte-identical")
