"""On-box peak measurements that bench.py divides by (the spec peaks re-measured on
the box): fcg_measure_peaks (STREAM triad, FP64 VALU, FP64 MFMA) and fcg_measure_hbm (16-byte copy,
write-only fill).  Plausibility bounds only: each figure positive and below the MI355X spec sheet
(8 TB/s HBM, 78.6 TF/s FP64), and the HBM patterns within a factor of two of each other."""
import importlib

import pytest

fcg = importlib.import_module("4c_amd").fcg

pytestmark = pytest.mark.gpu

HBM_SPEC_GBS = 8000.0
FP64_SPEC_TFS = 78.6


def test_measured_peaks_are_plausible():
    triad, valu, mfma = fcg.measure_peaks(0)
    copy, write = fcg.measure_hbm(0)
    for gbs in (triad, copy, write):
        assert 500.0 < gbs < HBM_SPEC_GBS * 1.05, (triad, copy, write)
    assert max(triad, copy, write) < 2.0 * min(triad, copy, write)
    for tfs in (valu, mfma):
        assert 1.0 < tfs < FP64_SPEC_TFS * 1.05, (valu, mfma)

