import cProfile, pstats, sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tensorcrossinterpolation.jl_amd"))
import tci_amd as T
f = T.quantics_osc(40)
p0 = T.optfirstpivot(f, [2] * 40)
T.crossinterpolate2(f, [2] * 40, [p0], tolerance=1e-8, nsearchglobalpivot=0, maxiter=1)
pr = cProfile.Profile(); pr.enable()
for _ in range(3):
    T.crossinterpolate2(f, [2] * 40, [p0], tolerance=1e-8, nsearchglobalpivot=0)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
