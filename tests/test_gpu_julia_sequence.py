"""GPU: the Julia binding's call sequence, replayed through ctypes.

julia/RBL_hip.jl (the `RBL_gpu(A,k,b)` drop-in for RBL_gpu.jl:205-221) cannot run here: Julia is
absent from the image.  tests/test_julia_binding.py checks each of its `ccall`s
against include/rbl_hip.h; this test drives the library exactly as that file's `RBL_hip` does —
the same entry points in the same order with the same argument conventions — so the conventions
only the Julia side uses are exercised on the device:

  * `rbl_set_matrix_csc` with Julia's 1-based Int64 `colptr` / `rowval` (index_base 1; the Python
    host passes 0-based arrays), or `rbl_set_matrix_dense` with the column-major matrix as-is;
  * `rbl_start` with a NULL Omega and a seed; `rbl_step_async` per step with the partial-reorth
    flag of RBL_gpu.jl:164; `rbl_fetch` into column-major b x b x m arrays (Julia's `Ah[:, :, j]`);
  * the host loop of RBL_hip.jl: the reference's own `insertA!` / `insertB!` / `dsbev` /
    `sort_eig_abs` / `check_convergence` (common.jl:9-65, here their restatement in
    oracle/rbl_oracle.py), its speculation rule, `D[end:-1:1]`, the sign fix, and `rbl_ritz`
    with S and V column-major.

Checked against the Python host (`rbl.lanczos`, 0-based CSC, rbl.host's eigensolver) with the same
seed: every A_i / B_{i+1} bit for bit (the device sees the same matrix and Omega), the same step
count, eigenvalues within 1e-12 relative (the reference's dsbev vs rbl.host's dsbevd), Ritz vectors
within 1e-9, residuals < 1e-7.  The restarted binding (`RBL_hip_restarted`, restarted.jl:106-146:
rbl_step with the restart flags, rbl_reorth_last, rbl_lock, rbl_restart, rbl_get_locked) is
replayed the same way against rbl.RBL_gpu_restarted: the same cycles, locked eigenvalues within
1e-9, locked vectors' residuals < 1e-7."""
import ctypes as C

import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def _julia_rbl_hip(rbl, A, k, b, seed, kryl_sz=1200):
    """RBL_hip(A, k, b; seed) of julia/RBL_hip.jl, line by line (comments: its statements)."""
    from rbl import _lib
    lib = _lib.lib
    n = A.shape[1]
    h = C.c_void_p()
    assert lib.rbl_create(C.byref(h), 0) == 0                       # rbl_context(device)
    steps_A, steps_B = [], []

    def check(st, what):
        if st < 0:
            raise AssertionError(f"{what}: {st} {lib.rbl_last_error(h)}")

    try:
        if isinstance(A, np.ndarray):                               # set_matrix!(ctx, ::Matrix)
            Af = np.asfortranarray(A, dtype=np.float64)
            check(lib.rbl_set_matrix_dense(h, n, 0, n, _lib.dptr(Af), n), "rbl_set_matrix_dense")
        else:                                                       # set_matrix!(ctx, ::SparseMatrixCSC)
            Cm = A.tocsc()
            Cm.sort_indices()
            colptr = Cm.indptr.astype(np.int64) + 1                 # Julia's 1-based arrays
            rowval = Cm.indices.astype(np.int64) + 1
            nzval = Cm.data.astype(np.float64)
            check(lib.rbl_set_matrix_csc(h, n, Cm.nnz, _lib.i64ptr(colptr), _lib.i64ptr(rowval),
                                         _lib.dptr(nzval), 1), "rbl_set_matrix_csc")
        check(lib.rbl_set_option(h, _lib.RBL_OPT_DEVICE_BLOCKS, 0), "rbl_set_option")
        check(lib.rbl_set_option(h, _lib.RBL_OPT_TIMERS, 0), "rbl_set_option")
        m_max = -(-kryl_sz // b)                                    # cld(kryl_sz, b)
        check(lib.rbl_start(h, b, m_max, 64, None, seed), "rbl_start")
        enq = [0]

        def enqueue(upto):
            while enq[0] < upto:
                enq[0] += 1
                part = 1 if enq[0] >= 2 and enq[0] % 2 == 0 else 0  # RBL_gpu.jl:164
                check(lib.rbl_step_async(h, enq[0], part), "rbl_step_async")

        def fetch(i0, i1):
            m = i1 - i0
            Ah = np.zeros((b, b, m), order="F")                     # zeros(Float64, b, b, m)
            Bh = np.zeros((b, b, m), order="F")
            sts = np.zeros(m, np.int32)
            check(lib.rbl_fetch(h, i0, i1, _lib.dptr(Ah), _lib.dptr(Bh), _lib.i32ptr(sts)),
                  "rbl_fetch")
            return Ah, Bh

        resid = []
        T = None
        D = V = None
        converged = False
        first, i = 1, 0
        while True:
            i += 1
            is_check = i >= 2 and i * b > k and i % 4 == 0
            is_last = not (i * b < kryl_sz and i < m_max)
            if not (is_check or is_last):
                continue
            enqueue(i)
            if is_check and not is_last and i % 2 == 0 and len(resid) >= 2 and resid[-1] > 0 \
                    and resid[-2] > 0:
                pred = resid[-1] * min(1.0, resid[-1] / resid[-2])
                ahead = 4 if pred > 100e-7 else 2 if pred > 5e-7 else 1 if pred > 1e-7 else 0
                enqueue(min(i + ahead, m_max))
            Ah, Bh = fetch(first, i + 1)
            for jj, j in enumerate(range(first, i + 1)):
                Ai, Bi = Ah[:, :, jj].copy(), Bh[:, :, jj].copy()
                steps_A.append(Ai)
                steps_B.append(Bi)
                slab = o.insertA(Ai, b)                              # insertA!(Ai, b)
                T = slab if j == 1 else np.hstack([T, slab])         # T = [T insertA!(Ai, b)]
                if j == i and is_check:
                    D, V = o.dsbev(T)                                # dsbev('V', 'L', T)
                    D, V = o.sort_eig_abs(D, V, k)
                    Y = Bi @ V[-b:, :]
                    resid.append(max(np.linalg.norm(Y[:, l]) for l in range(k)))
                    if o.check_convergence(Bi, V, b, k, 1e-7):
                        converged = True
                        break
                o.insertB(Bi, T, b, j)                               # insertB!(Bi, T, b, j)
            first = i + 1
            if converged or is_last:
                break
        D = D[::-1].copy()                                           # D[end:-1:1]
        S = np.asfortranarray(V[:, ::-1])
        for c in range(S.shape[1]):                                  # the sign fix
            p = int(np.argmax(np.abs(S[:, c])))
            if S[p, c] < 0:
                S[:, c] *= -1
        nblocks = S.shape[0] // b
        Vout = np.zeros((n, k), order="F")
        check(lib.rbl_ritz(h, nblocks, k, _lib.dptr(S), _lib.dptr(Vout)), "rbl_ritz")
        return D, Vout, i, converged, steps_A, steps_B
    finally:
        lib.rbl_free(h)


@pytest.mark.parametrize("kind", ["sparse", "dense"])
def test_julia_call_sequence_matches_python_host(rbl, kind):
    k, b, seed = 10, 8, 20261018
    if kind == "sparse":
        A = matgen.hashwindow_csr(6000, 48, 0.5, 11, matgen.planted_spectrum(k))
    else:
        A = matgen.hashwindow_csr(1500, 300, 0.3, 5, matgen.planted_spectrum(k)).toarray()
    D, V, iters, converged, tA, tB = _julia_rbl_hip(rbl, A, k, b, seed)
    assert converged
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        Dp, Vp, info = rbl.lanczos(ctx, k, b, seed=seed, trace=True)
    assert info.converged and info.iters == iters
    # the same device computation: A_i / B_{i+1} bit for bit (fetch's column-major layout and
    # the 1-based matrix upload change nothing the device computes)
    assert len(tA) >= info.iters and len(info.trace_A) == info.iters
    for j in range(info.iters):
        assert np.array_equal(tA[j], info.trace_A[j]), j
        assert np.array_equal(tB[j], info.trace_B[j]), j
    assert np.all(np.abs(D - Dp) <= 1e-12 * np.abs(Dp)), np.abs(D - Dp) / np.abs(Dp)
    assert np.abs(V - Vp).max() < 1e-9
    res = np.linalg.norm(A @ V - V * D, axis=0) / np.abs(D)
    assert res.max() < 1e-7


def _julia_rbl_hip_restarted(A, k, seed, kryl0=100, max_cycles=60):
    """RBL_hip_restarted(A, k; seed) of julia/RBL_hip.jl (restarted.jl:106-146), line by line."""
    from rbl import _lib
    lib = _lib.lib
    n = A.shape[1]
    b = 1
    h = C.c_void_p()
    assert lib.rbl_create(C.byref(h), 0) == 0

    def check(st, what):
        if st < 0:
            raise AssertionError(f"{what}: {st} {lib.rbl_last_error(h)}")

    try:
        Cm = A.tocsc()
        Cm.sort_indices()
        colptr = Cm.indptr.astype(np.int64) + 1
        rowval = Cm.indices.astype(np.int64) + 1
        nzval = Cm.data.astype(np.float64)
        check(lib.rbl_set_matrix_csc(h, n, Cm.nnz, _lib.i64ptr(colptr), _lib.i64ptr(rowval),
                                     _lib.dptr(nzval), 1), "rbl_set_matrix_csc")
        check(lib.rbl_start(h, b, kryl0 + 10 * max_cycles, 64, None, seed), "rbl_start")
        Ai = np.zeros((b, b), order="F")
        Bi = np.zeros((b, b), order="F")

        def step(i, flags):
            check(lib.rbl_step(h, i, flags, _lib.dptr(Ai), _lib.dptr(Bi)), "rbl_step")

        D = []
        count, kryl, cycles = 0, kryl0, 0
        while count < k and cycles < max_cycles:
            step(1, 2)                                               # :41-50
            T = o.insertA(Ai.copy(), b)
            o.insertB(Bi.copy(), T, b, 1)
            i = 2
            while i * b < kryl:                                      # :52-86
                step(i, 3 if i % 3 == 0 else 0)
                T = np.hstack([T, o.insertA(Ai.copy(), b)])
                if (i + 1) * b < kryl:
                    o.insertB(Bi.copy(), T, b, i)
                i += 1
            m = i - 1
            check(lib.rbl_reorth_last(h, m, 3), "rbl_reorth_last")  # :100-102
            d, v = o.dsbev(T)                                        # :103
            conv = Bi @ v[-b:, ::-1]                                 # :104
            d, v = d[::-1], v[:, ::-1]
            ncomp, restart = 0, None
            for j in range(d.size):                                  # :116-137
                if count + ncomp >= k:
                    break
                if np.linalg.norm(conv[:, j]) < 1e-7:
                    ncomp += 1
                    s = np.asfortranarray(v[:, j:j + 1])      # Julia's v[:, j:j]
                    check(lib.rbl_lock(h, m, 1, _lib.dptr(s)), "rbl_lock")
                    D.append(float(d[j]))
                else:
                    restart = np.asfortranarray(v[:, j:j + 1])
                    break
            if restart is None:
                restart = np.zeros((m * b, b), order="F")
                restart[0, 0] = 1.0
            check(lib.rbl_restart(h, m, _lib.dptr(restart)), "rbl_restart")
            kryl += 10
            count += ncomp
            cycles += 1
        L = lib.rbl_num_locked(h)
        V = np.zeros((n, L), order="F")
        if L > 0:
            check(lib.rbl_get_locked(h, _lib.dptr(V)), "rbl_get_locked")
        return np.asarray(D), V, cycles
    finally:
        lib.rbl_free(h)


def test_julia_restarted_call_sequence_matches_python_host(rbl):
    """RBL_hip_restarted's sequence (rbl_step with the restart flags, rbl_reorth_last, rbl_lock,
    rbl_restart, rbl_get_locked) on a 1-based CSC upload against rbl.RBL_gpu_restarted with the
    same seed: the same cycles, locked eigenvalues within 1e-9 relative, locked vectors' residuals
    < 1e-7 (the tolerances of test_gpu_restarted.py)."""
    k, seed = 5, 77
    A = matgen.hashwindow_csr(3000, 40, 0.5, 3, matgen.planted_spectrum(k))
    D, V, cycles = _julia_rbl_hip_restarted(A, k, seed)
    Dp, Vp, cyc_p = rbl.RBL_gpu_restarted(A, k, seed=seed, return_cycles=True)
    assert cycles == cyc_p and D.size == Dp.size == k
    assert np.all(np.abs(D - Dp) <= 1e-9 * np.abs(Dp)), (D, Dp)
    res = np.linalg.norm(A @ V - V * D[None, :], axis=0) / np.abs(D)
    assert res.max() < 1e-7, res


@pytest.mark.parametrize("b", [8, 32])
def test_unsymmetric_A_multiplies_by_A(rbl, b):
    """An unsymmetric A (benchmark.jl:58 runs RBL_gpu on an unsymmetric sprandn; cuSPARSE then
    multiplies by A itself): the Python host uploads A's rows and julia/RBL_hip.jl uploads the
    CSC arrays of A^T, 1-based — both make rbl_apply compute A X (not A^T X), within
    1e-13 |A||X| of SciPy, and the two uploads give the same Y bit for bit."""
    import scipy.sparse as sp
    from rbl import _lib
    lib = _lib.lib
    n = 3000
    A = sp.random(n, n, density=0.01, random_state=5, format="csr") + sp.diags(np.arange(1.0, n + 1))
    A = sp.csr_matrix(A)
    X = np.asfortranarray(np.random.default_rng(2).standard_normal((n, b)))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        Y = ctx.apply(X)
    ref = A @ X
    assert np.all(np.abs(Y - ref) <= 1e-13 * (abs(A) @ np.abs(X)) + 1e-300)
    assert np.abs(Y - A.T @ X).max() > 1e-3 * np.abs(ref).max()   # A is far from symmetric
    Ct = sp.csc_matrix(A.T)                         # SparseMatrixCSC(transpose(A))
    Ct.sort_indices()
    colptr = Ct.indptr.astype(np.int64) + 1
    rowval = Ct.indices.astype(np.int64) + 1
    nzval = Ct.data.astype(np.float64)
    h = C.c_void_p()
    assert lib.rbl_create(C.byref(h), 0) == 0
    try:
        assert lib.rbl_set_matrix_csc(h, n, Ct.nnz, _lib.i64ptr(colptr), _lib.i64ptr(rowval),
                                      _lib.dptr(nzval), 1) == 0
        Yj = np.zeros((n, b), order="F")
        assert lib.rbl_apply(h, b, _lib.dptr(X), _lib.dptr(Yj)) == 0
    finally:
        lib.rbl_free(h)
    assert np.array_equal(Yj, Y)
