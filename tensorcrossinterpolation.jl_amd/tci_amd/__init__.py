"""tci_amd -- MI355X-native TCI2 hot path for TensorCrossInterpolation.jl.

Host-side mirror of the reference's API for the path this package replaces (rrlu / MatrixLUCI /
batch evaluation / TensorCI2 / crossinterpolate2); all compute runs in libtci_hip.so (gfx950).
"""
from ._lib import Context, TCIArgumentError, TCIDeviceError, TCIError, context, load
from .batcheval import (ComplexScaledEvaluator, F_CP, F_GAUSS, F_GAUSSMIX, F_LORENTZ, F_MPO, F_QEXP, F_QOSC, F_SUM, F_TABLE, F_TT,
                        GPUBatchEvaluator, cp_function, gauss, gaussmix, lorentz, quantics_bits,
                        quantics_exp, quantics_osc, sum_, table, tensortrain_function)
from .cachedfunction import CachedFunction
from .contraction import Contraction, contract, contract_naive, contract_TCI
from .distributed import (Comm, DeviceComm, HostExchange, ShardedBatchEvaluator, column_blocks, rrlu_sharded,
                          rrlu_sharded_factors)
from .hostfunction import HostFunctionEvaluator
from .globalpivotfinder import AbstractGlobalPivotFinder, DefaultGlobalPivotFinder, FixedGlobalPivotFinder
from .matrixlu import (DeviceMatrix, colindices, dgemm_device, diag, lastpivoterror, ldiv, left, npivots,
                       pivoterrors, right, rowindices, rrLU, rrlu, rrlu_inplace_device, schur_update_device,
                       sitetensor_solve_device)
from .matrixluci import MatrixLUCI
from .tensorci2 import (TensorCI2, convergencecriterion, crossinterpolate2, forwardsweep, kronecker_left, optfirstpivot,
                        kronecker_right, union_sets)

__all__ = [name for name in dir() if not name.startswith("_")]
