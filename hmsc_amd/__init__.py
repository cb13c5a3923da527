"""hmsc_amd — MI355X-native Gibbs sampler behind Hmsc's ``sampleMcmc()``.

Host API mirroring the reference R package (taddallas/HMSC, Hmsc 3.0-4):
``Hmsc``, ``HmscRandomLevel``, ``setPriors``, ``sampleMcmc``,
``convertToCodaObject``, ``alignPosterior``, ``computeWAIC`` ...; the per-sweep
hot path runs as hand-written HIP kernels for gfx950 in ``libhmsc_amd.so``
behind the C ABI ``include/hmsc_amd.h``.
"""
from .model import Hmsc, HmscRandomLevel, setPriors, model_matrix  # noqa: F401
from .post import (computeAssociations, computeVariancePartitioning, convertToCodaObject, computeWAIC, effectiveSize,  # noqa: F401
                   gelman_diag, getPostEstimate, poolMcmcChains, spectrum0_ar)
from .sampler import Chain, alignPosterior, combine_parameters, sampleMcmc, updater_mask  # noqa: F401
from .dataparams import computeDataParameters, constructKnots  # noqa: F401
from .predict import computePredictedValues, evaluateModelFit, predict, predictLatentFactor  # noqa: F401

__all__ = ["Hmsc", "HmscRandomLevel", "setPriors", "sampleMcmc", "convertToCodaObject", "computeWAIC",
           "effectiveSize", "gelman_diag", "getPostEstimate", "poolMcmcChains", "alignPosterior",
           "computeDataParameters", "constructKnots", "Chain", "computeVariancePartitioning", "predict", "predictLatentFactor",
           "computePredictedValues", "evaluateModelFit"]
