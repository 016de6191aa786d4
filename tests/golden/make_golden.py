"""Writes tests/golden/reference_kats.json: the known-answer tests (KATs) that the reference
ships for the TCI2 hot path, as data (input matrices + the outcome each reference test asserts).

Sources (all in /root/reference, read as text; Julia is absent, so nothing was executed):
  test/test_matrixlu.jl   :8-29 (argmax 10x8), :39-52 (complex 3x6), :54-69 (exact 4x4),
                           :88-97 (rank-1 truncation), :99-139 (8x6 maxrank 4 / reltol 1e-2),
                           :141-165 (exact rank 3), :167-175 (pivoterrors [1,1,0]),
                           :177-195 (maxrank/abstol 5x5), :197-211 (1e-13 scaled, abstol)
  test/test_matrixluci.jl :6-74 (LUCI vs MatrixCI inverse; exact low rank; cond < 1e12)
  test/test_batcheval.jl  :13-35 (M=1 / M=2 closed forms with f = sum)
  test/test_tensorci2.jl  :9-25 (kronecker), :27-39 (pivoterrors == [1, 1e-5, 0]),
                           :247-339 (Lorentz 5d), :504-554 (convergencecriterion truth table)
  test/test_integration.jl:29-37 (Iref = -5.4960415218049, used as a documented target only)

Expected values that the reference test states as a property (e.g. `npivots(lu) == 3`) are
stored as that property; tests/test_oracle_kats.py checks the oracle against every entry.
Run: python tests/golden/make_golden.py
"""
import json
import os

A_10x8 = [
    [0.0698159, 0.334367, -0.589437, 0.145762, 0.812079, -0.756145, 0.295355, 0.474037],
    [0.700284, 0.53583, -0.879161, 0.0259543, -0.17721, 0.872417, -0.130773, 0.806836],
    [-0.27785, 0.75619, -0.6596, 0.697439, 0.751422, -0.694813, 0.5158, -0.812036],
    [-0.621557, 0.183863, -0.163899, -0.0200506, 0.418512, 0.456449, 0.779305, 0.771141],
    [-0.71849, -0.343808, 0.360291, 0.311619, -0.609726, 0.309062, -0.214459, -0.830421],
    [-0.320604, -0.998123, 0.45783, 0.990825, -0.790207, -0.227163, -0.535666, -0.950299],
    [-0.136987, -0.0648093, -0.960298, 0.454315, -0.722124, 0.782378, 0.356427, 0.987233],
    [-0.209571, -0.0171136, 0.189971, 0.578491, -0.663334, -0.482773, -0.0205025, 0.570071],
    [-0.942577, 0.306031, 0.696775, -0.853113, 0.554776, -0.25695, 0.229594, -0.0306027],
    [-0.490229, -0.0501003, 0.163198, -0.253586, 0.941586, 0.0345018, 0.737874, -0.963045],
]

A_4x4 = [
    [0.711002, 0.724557, 0.789335, 0.382373],
    [0.910429, 0.726781, 0.719957, 0.486302],
    [0.632716, 0.39967, 0.571809, 0.0803125],
    [0.885709, 0.531645, 0.569399, 0.481214],
]

A_8x6 = [
    [0.684025, 0.784249, 0.826742, 0.054321, 0.0234695, 0.467096],
    [0.73928, 0.295516, 0.877126, 0.111711, 0.103509, 0.653785],
    [0.394016, 0.753239, 0.889128, 0.291669, 0.873509, 0.0965536],
    [0.378539, 0.0123737, 0.20112, 0.758088, 0.973042, 0.308372],
    [0.235156, 0.51939, 0.788184, 0.363171, 0.230001, 0.984971],
    [0.893223, 0.220834, 0.18001, 0.258537, 0.396583, 0.142105],
    [0.0417881, 0.890706, 0.328631, 0.279332, 0.963188, 0.706944],
    [0.914298, 0.792345, 0.311083, 0.129653, 0.350062, 0.683966],
]

# test_matrixluci.jl:7-16 differs from the rrLU test in one digit (0.46709 vs 0.467096)
A_8x6_luci = [row[:] for row in A_8x6]
A_8x6_luci[0][5] = 0.46709

P_10x3 = [
    [0.284975, 0.505168, 0.570921],
    [0.302884, 0.475901, 0.645776],
    [0.622955, 0.361755, 0.99539],
    [0.748447, 0.354849, 0.431366],
    [0.28338, 0.0378148, 0.994162],
    [0.643177, 0.74173, 0.802733],
    [0.58113, 0.526715, 0.879048],
    [0.238002, 0.557812, 0.251512],
    [0.458861, 0.141355, 0.0306212],
    [0.490269, 0.810266, 0.7946],
]
Q_3x10 = [
    [0.239552, 0.306094, 0.299063, 0.0382492, 0.185462, 0.0334971, 0.697561, 0.389596, 0.105665, 0.0912763],
    [0.0570609, 0.56623, 0.97183, 0.994184, 0.371695, 0.284437, 0.993251, 0.902347, 0.572944, 0.0531369],
    [0.45002, 0.461168, 0.6086, 0.613702, 0.543997, 0.759954, 0.0959818, 0.638499, 0.407382, 0.482592],
]

A_5x5 = [
    [0.433088, 0.956638, 0.0907974, 0.0447859, 0.0196053],
    [0.855517, 0.782503, 0.291197, 0.540828, 0.358579],
    [0.37455, 0.536457, 0.205479, 0.75896, 0.701206],
    [0.47272, 0.0172539, 0.518177, 0.242864, 0.461635],
    [0.0676373, 0.450878, 0.672335, 0.77726, 0.540691],
]

A_tiny = [
    [0.585383, 0.124568, 0.352426, 0.573507],
    [0.865875, 0.600153, 0.727443, 0.902388],
    [0.913477, 0.954081, 0.116965, 0.817],
    [0.985918, 0.516114, 0.600366, 0.0200085],
]

kats = {
    "source": "XiaoJiang-Phy/TensorCrossInterpolation.jl test/ (see make_golden.py docstring)",
    "argmax_10x8": {
        "A": A_10x8,
        "ref": "test_matrixlu.jl:8-29",
        # identity f; expectations restated from Julia argmax (column-major first max)
        "cases": [
            {"rows": [3], "cols": [5], "expect": [3, 5]},
            {"rows": ":", "cols": ":", "expect": "argmax(A)"},
            {"rows": [1], "cols": ":", "expect": "(1, argmax(A[1,:]))"},
            {"rows": ":", "cols": [1], "expect": "(argmax(A[:,1]), 1)"},
            {"start": 1, "expect": "argmax(A)"},
            {"start": 8, "expect": [8, 8]},
        ],
    },
    "argmax_complex_3x6": {
        "ref": "test_matrixlu.jl:39-52; abs2 of the complex entries (|z|^2 is real)",
        "note": "row 2 is `1 +im 2+im ...` = [1, im, 2+im, 3+im, 4+im, 5+im] in Julia's "
                "space-separated matrix literal (unary +im is its own element)",
        "re": [[0, 1, 2, 3, 4, 5], [1, 0, 2, 3, 4, 5], [1, 0, 2, 3, 4, 5]],
        "im": [[0, 0, 0, 0, 0, 0], [0, 1, 1, 1, 1, 1], [0, 2, 2, 2, 2, 2]],
        "cases": [
            {"rows": [3], "cols": [5], "expect": [3, 5]},
            {"rows": ":", "cols": ":", "expect": "argmax(abs2.(A))"},
            {"rows": [1], "cols": ":", "expect": "(1, argmax(abs2.(A[1,:])))"},
            {"rows": ":", "cols": [1], "expect": "(argmax(abs2.(A[:,1])), 1)"},
            {"start": 1, "expect": "argmax(abs2.(A))"},
        ],
    },
    "argmax_throws": {
        "ref": "test_matrixlu.jl:31-37",
        "cases": [
            {"n": 10, "start": 100, "error": "rows must not be empty"},
            {"n": 10, "rows": [3], "cols": [], "error": "cols must not be empty"},
            {"n": 10, "rows": [1, 100, 1000], "cols": [1], "error": "rows"},
            {"n": 10, "rows": [1], "cols": [1, 100, 1000], "error": "cols"},
        ],
    },
    "rrlu_exact_4x4": {"A": A_4x4, "ref": "test_matrixlu.jl:54-69",
                        "expect": {"unit_lower_L": True, "upper_U": True, "reconstruct_rtol": 1.49e-8}},
    "rrlu_truncated_rank1": {"A": [[1.0, 0, 0], [0, 0, 0], [0, 0, 0]], "ref": "test_matrixlu.jl:88-97",
                              "expect": {"npivot": 1}},
    "rrlu_maxrank4_8x6": {"A": A_8x6, "ref": "test_matrixlu.jl:99-120",
                           "kwargs": {"maxrank": 4},
                           "expect": {"npivot": 4, "L_shape": [8, 4], "U_shape": [4, 6],
                                      "tril_L": True, "triu_U": True}},
    "rrlu_reltol_8x12": {"A": A_8x6, "ref": "test_matrixlu.jl:122-138",
                          "note": "A = hcat(A, A .+ 1e-3*rand(8,6)); Julia's rand is not reproducible "
                                  "here, the perturbation is regenerated with numpy seed 0",
                          "kwargs": {"reltol": 1e-2},
                          "expect": {"rank_below": [8, 12], "max_abs_residual_below": 1e-2}},
    "rrlu_exact_rank3": {"p": P_10x3, "q": Q_3x10, "ref": "test_matrixlu.jl:141-165",
                          "expect": {"npivot": 3, "reconstruct_rtol": 1.49e-8}},
    "rrlu_identity_pivoterrors": {"A": [[1.0, 0.0], [0.0, 1.0]], "ref": "test_matrixlu.jl:167-175",
                                   "expect": {"pivoterrors": [1.0, 1.0, 0.0], "lastpivoterror": 0.0}},
    "rrlu_limits_5x5": {"A": A_5x5, "ref": "test_matrixlu.jl:177-195",
                         "cases": [
                             {"kwargs": {"maxrank": 2}, "expect": {"n_pivoterrors": 3, "lastpivoterror_gt": 0.0}},
                             {"kwargs": {"abstol": 0.5}, "expect": {"lastpivoterror_lt": 0.5}},
                             {"kwargs": {"abstol": 0.0}, "expect": {"lastpivoterror": 0.0}},
                         ]},
    "rrlu_tiny_values": {"A": A_tiny, "scale": 1e-13, "ref": "test_matrixlu.jl:197-211",
                          "kwargs": {"abstol": 1e-3},
                          "expect": {"npivot": 1, "lastpivoterror_gt": 0.0, "max_abs_residual_below": 1e-3}},
    "luci_maxrank4_8x6": {"A": A_8x6_luci, "ref": "test_matrixluci.jl:6-37",
                           "kwargs": {"maxrank": 4},
                           "expect": {"left_eq_C_Pinv": True, "right_eq_Pinv_R": True, "rtol": 1.49e-8}},
    "luci_exact_rank3": {"p": P_10x3, "q": Q_3x10, "ref": "test_matrixluci.jl:48-74",
                          "expect": {"npivot": 3, "reconstruct_rtol": 1.49e-8, "cond_pivot_below": 1e12}},
    "batcheval_sum": {"ref": "test_batcheval.jl:13-35",
                      "cases": [
                          {"localdims": [2, 2, 2, 2, 2], "left": [[1, 1]], "right": [[1, 1]], "M": 1,
                           "expect": "sum(vcat(l, c, r))"},
                          {"localdims": [2, 2, 2, 2, 2], "left": [[1]], "right": [[1, 1]], "M": 2,
                           "expect": "sum(vcat(l, c, cp, r))"},
                      ]},
    "kronecker": {"ref": "test_tensorci2.jl:9-25", "multiset": [[1, 2, 3, 4, 5]] * 5, "localdim": 4},
    "tci2_pivoterrors": {"ref": "test_tensorci2.jl:27-39",
                          "f": "x[1]==x[2] ? diags[x[1]] : 0", "diags": [1.0, 1e-5, 0.0],
                          "localdims": [3, 3], "initialpivots": [[1, 1]], "tolerance": 1e-8,
                          "expect": {"pivoterrors": [1.0, 1e-5, 0.0]}},
    "tci2_lorentz5d": {"ref": "test_tensorci2.jl:247-339",
                        "f": "coeff / (sum(v.^2) + 1)", "coeff": 1.0, "n": 5, "d": 10,
                        "updatepivots_maxbonddim2": {"reltol": 1e-8, "expect_linkdims": [2, 2, 2, 2]},
                        "globalpivot": [2, 9, 10, 5, 7],
                        "after_global_1site": {"reltol": 1e-12, "expect_linkdims": [3, 3, 3, 3]},
                        "crossinterpolate2_tol1e-12": {"maxiter": 200, "expect_pivoterror_le": 2e-12,
                                                       "expect_rank_le": 200},
                        "initialpivots_5": [[1, 1, 1, 1, 1], [10, 8, 10, 4, 4], [5, 4, 8, 9, 3],
                                            [7, 7, 10, 5, 9], [7, 7, 10, 5, 9]],
                        "eval_grid": 3},
    "convergencecriterion": {"ref": "test_tensorci2.jl:504-554",
                             "cases": [
                                 {"ranks": [1, 2], "errors": [1e-2, 1e-5], "ngp": [0, 0], "tol": 1e-4,
                                  "maxbonddim": 4, "ncheck": 3, "expect": False},
                                 {"ranks": [1, 2, 2, 2], "errors": [1e-2, 1e-5, 1e-5, 1e-5], "ngp": [0, 0, 0, 0],
                                  "tol": 1e-4, "maxbonddim": 4, "ncheck": 3, "expect": True},
                                 {"ranks": [1, 2, 2, 2], "errors": [1e-2, 1e-2, 1e-5, 1e-5], "ngp": [0, 0, 0, 0],
                                  "tol": 1e-4, "maxbonddim": 4, "ncheck": 3, "expect": False},
                                 {"ranks": [1, 2, 2, 2], "errors": [1e-2, 1e-2, 1e-2, 1e-2], "ngp": [0, 0, 0, 0],
                                  "tol": 1e-4, "maxbonddim": 2, "ncheck": 3, "expect": True},
                                 {"ranks": [1, 2, 2, 2], "errors": [1e-2, 1e-2, 1e-2, 1e-2], "ngp": [0, 1, 1, 1],
                                  "tol": 1e-4, "maxbonddim": 2, "ncheck": 3, "expect": True},
                             ]},
    "quantics_exp_trivial": {"ref": "test_tensorci2.jl:55-102 (nsearchglobalpivot=0, :full)",
                              "R": 8, "abstol": 1e-4, "maxbonddim": 1, "maxiter": 2,
                              "firstpivots": [[1] * 8, [1] + [2] * 7],
                              "x_points": [0.1, 0.3, 0.6, 0.9],
                              "expect": {"linkdims_all": 1, "abs_err_below": 1e-4}},
    "integrate_10d": {"ref": "test_integration.jl:29-37", "Iref": -5.4960415218049, "tol": 1e-3,
                      "note": "documented end-to-end target; integration is a caller of the hot path "
                              "and out of scope for this round"},
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as fh:
        json.dump(kats, fh, indent=1)
    print("wrote", out)
