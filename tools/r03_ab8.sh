# Round-3 A/B 8: fp32-basis Gram k_gram32 — 8-B basis loads (RBL_G32_W8) and MFMA accumulators
# in arch VGPRs (-mllvm -amdgpu-mfma-vgpr-form for reorth32.hip) — tree vs tools/variants/f32base
# (neither) and tools/variants/w8novgpr (loads only).  fp32 tests, bit identity, probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp32_basis.py tests/test_gpu_c5.py tests/test_gpu_spill.py > gpurun_out/r03_ab8_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab8_tests.log
[ $rc -ne 0 ] && exit $rc
cat > gpurun_out/bit32.py <<'PY'
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.getcwd(), "gpu-randomized-block-lanczos_amd"))
import scipy.sparse as sp
import rbl
out = {}
for n in (3001, 20000):
    R = sp.random(n, n, density=min(0.004, 40.0 / n), random_state=5, format="csr")
    A = (R + R.T + sp.diags(np.linspace(1.0, 3.0, n))).tocsr()
    for b in (16, 32):
        omega = np.random.default_rng(b).standard_normal((n, b))
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            D, V, info = rbl.lanczos(ctx, 10, b, omega=omega, max_steps=14, trace=True, basis_bits=32)
        out[f"D_{n}_{b}"] = np.asarray(D)
        out[f"V_{n}_{b}"] = np.asarray(V, dtype=np.float64)
        out[f"A_{n}_{b}"] = np.concatenate([np.ravel(x) for x in info.trace_A])
np.savez(sys.argv[1], **out)
PY
timeout -k 10 300 python gpurun_out/bit32.py gpurun_out/b32_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/f32base/librbl_hip.so timeout -k 10 300 python gpurun_out/bit32.py gpurun_out/b32_base.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/b32_tree.npz gpurun_out/b32_base.npz
rm -f gpurun_out/b32_*.npz
for rep in 1 2; do
  for v in f32base w8novgpr tree; do
    echo "== $v (rep $rep)"
    if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
    timeout -k 10 120 ./tools/reorth32_probe | tail -2 || exit 1
  done
done
