"""Build slate_amd's native host module with AddressSanitizer + UBSan into
<outdir>/slate_amd_asan/_host.so and run host kernels against it in a child
interpreter with libasan preloaded (sanitizer configuration of
the host code).  Exit 77 = toolchain lacks libasan (skip)."""
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out):
    asan = subprocess.run(["g++", "-print-file-name=libasan.so"], stdout=subprocess.PIPE, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        print("no libasan")
        return 77
    import pybind11
    inc = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
           "-I" + os.path.join(ROOT, "slate_amd", "csrc", "include")]
    pkg = os.path.join(out, "asanpkg")
    os.makedirs(pkg, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "slate_amd", "csrc", "host", "*.cpp")))
    so = os.path.join(pkg, "_host.so")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"] + inc + srcs + ["-o", so]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode:
        print(r.stdout)
        return 1
    child = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
import slate_amd._native as N                # SLATE_AMD_HOST_LIB: every host kernel runs in the ASan build
assert N._host.__file__.endswith("asanpkg/_host.so"), N._host.__file__
from slate_amd import ops
import slate_amd as sl
torch.manual_seed(0)
for n, nb in ((50, 16), (97, 32)):
    A = sl.Matrix(n, n, nb=nb); A.insertLocalTiles(); sl.generate_matrix(A, "rands", 1)
    piv = sl.Pivots(); assert sl.getrf(A, piv) == 0
    H2 = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb); H2.insertLocalTiles(); sl.generate_matrix(H2, "poev", 2)
    assert sl.potrf(H2) == 0
    Q = sl.Matrix(n + 20, n, nb=nb); Q.insertLocalTiles(); sl.generate_matrix(Q, "rands", 3)
    T = sl.TriangularFactors(); sl.geqrf(Q, T)
    E = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb); E.insertLocalTiles(); sl.generate_matrix(E, "rands", 4)
    Z = sl.Matrix(n, n, nb=nb); Z.insertLocalTiles()
    sl.heev(E, None, Z)
    ipiv = torch.tensor([3, 1, 4, 7, 5], dtype=torch.int64)
    plan = ops.swap_plan(ipiv, 0, 5, 0)
    X = ops.colmajor_empty(10, 6, torch.float64, "cpu")
    B = torch.randn(6, 12, dtype=torch.float64).t()
    ops.xchg_gather(plan, B, X, 4, 1, 0); ops.xchg_scatter(plan, X, B, 4, 1, 0)
print("ASAN-OK")
'''
    env = dict(os.environ, LD_PRELOAD=asan, SLATE_AMD_HOST_LIB=so, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2",
               SLATE_AMD_HB2ST_THREADS="2")
    r = subprocess.run([sys.executable, "-c", child, ROOT, pkg], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=800)
    print(r.stdout[:3000] + ("\n...\n" + r.stdout[-1500:] if len(r.stdout) > 4500 else r.stdout[3000:]))
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/slate_amd_asan"))
