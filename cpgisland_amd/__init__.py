"""cpgisland_amd — MI355X-native hot path of CpGIslandFinder (ErangaD/CpGIsland).

Two data-parallel stages of /root/reference/CpGIslandFinder.java, built as HIP kernels
behind a C-ABI (include/cpg.h, libcpg.so):
  * training pass: Baum-Welch E-step expected counts (the MapReduce mapper behind
    BaumWelchDriver.runBaumWelchMR, :200) + labelled int64 transition/emission counts;
  * decode: exact Viterbi (HmmEvaluator.decode, :260) + island scan/filter (:262-339).
"""
from ._lib import CpgError, CpgInvalid  # noqa: F401  (fails loudly if libcpg.so is absent)
from .hmm import Context, HmmEvaluator, HmmModel  # noqa: F401

__all__ = ["CpgError", "CpgInvalid", "Context", "HmmEvaluator", "HmmModel"]
