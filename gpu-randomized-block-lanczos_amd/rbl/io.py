"""Matrix loaders for the inputs the reference's benchmark uses.

Julia/benchmark.jl:21-28 reads matrices with MatrixMarket.jl (`mmread("../Matrix/hood.mtx")`)
and MAT.jl (`matopen(...ldoor.mat)`, `read(file, "Problem")["A"]`, the SuiteSparse layout).
These return a SciPy CSC matrix of float64 — the SparseMatrixCSC{Float64,Int64} that
RBL_gpu(A, k, b) takes — ready for `Context.set_matrix` / `RBL_gpu`.  Host-side only.
"""
from __future__ import annotations

import os

import numpy as np
import scipy.io
import scipy.sparse as sp


def _finish(A, path: str, check_symmetric: bool):
    A = sp.csc_matrix(A, dtype=np.float64)
    if A.shape[0] != A.shape[1]:
        raise ValueError(f"{path}: matrix is {A.shape[0]} x {A.shape[1]}, not square")
    A.sum_duplicates()
    A.sort_indices()
    if check_symmetric:
        D = abs(A - A.T)
        scale = abs(A).max() if A.nnz else 0.0
        if D.nnz and D.max() > 1e-12 * max(scale, 1.0):
            raise ValueError(f"{path}: matrix is not symmetric (RBL needs A = A^T)")
    return A


def load_matrix_market(path: str, check_symmetric: bool = True) -> sp.csc_matrix:
    """`mmread(path)` (MatrixMarket.jl): coordinate real/integer/pattern, general or
    symmetric storage (symmetric files are expanded to both triangles)."""
    return _finish(scipy.io.mmread(path), path, check_symmetric)


def load_mat(path: str, key: str | None = None, check_symmetric: bool = True) -> sp.csc_matrix:
    """MATLAB v5 .mat (MAT.jl `matopen`/`read`): a SuiteSparse `Problem` struct (its field
    `A`), or the variable `key`, or the first sparse variable in the file.  (v7.3/HDF5 files
    need h5py, which this image does not ship.)"""
    m = scipy.io.loadmat(path, squeeze_me=True, struct_as_record=False)
    if key is not None:
        obj = m[key]
    elif "Problem" in m:
        obj = m["Problem"].A
    else:
        cands = [v for k, v in m.items() if not k.startswith("__") and sp.issparse(v)]
        if not cands:
            raise ValueError(f"{path}: no sparse matrix variable")
        obj = cands[0]
    return _finish(obj, path, check_symmetric)


def load_matrix(path: str, **kw) -> sp.csc_matrix:
    """Dispatch on the extension: .mtx / .mtx.gz (Matrix Market) or .mat."""
    base = path[:-3] if path.endswith(".gz") else path
    ext = os.path.splitext(base)[1].lower()
    if ext == ".mtx":
        return load_matrix_market(path, **kw)
    if ext == ".mat":
        return load_mat(path, **kw)
    raise ValueError(f"{path}: unknown matrix format (want .mtx or .mat)")
