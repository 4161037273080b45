"""MI355X-native bootstrap-inference engine for Oaxaca-Blinder decomposition.

Drop-in for the bootstrap driver of ``OaxacaBuilder::run()`` in dot-comma-hyphen/oaxaca-blinder-rs.
Import with ``importlib.import_module("oaxaca-blinder-rs_amd")`` (the directory name carries a
hyphen). See DESIGN.md for the kernels and INTEGRATION.md for the Rust/C binding.
"""
from . import _native
from ._native import OaxacaError
from .api import (BudgetAdjustment, ComponentResult, DecompositionDetail, OaxacaBlinder, OaxacaBuilder,
                  OaxacaResults, PreparedRun, QuantileDecompositionBuilder, QuantileDecompositionDetail,
                  QuantileDecompositionResults, ReferenceCoefficients, TwoFoldResults, parse_formula)
from .engine import Panel, aggregate, boot_multi, bootstrap_stats, rif, row_layout
from .frame import Frame, read_csv

__all__ = [
    "OaxacaBuilder", "OaxacaBlinder", "OaxacaResults", "TwoFoldResults", "DecompositionDetail",
    "ComponentResult", "BudgetAdjustment", "ReferenceCoefficients", "OaxacaError", "PreparedRun",
    "Panel", "boot_multi", "Frame", "read_csv", "aggregate", "bootstrap_stats", "rif", "row_layout", "parse_formula",
    "QuantileDecompositionBuilder", "QuantileDecompositionDetail", "QuantileDecompositionResults",
]
