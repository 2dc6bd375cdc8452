"""The shipped offline-tuned GEMM table (tuning/tunableop_mi355x.csv) only names solutions that
compute the right product without reading outside their operands (ops/gemm_tuning.py
check_tuned_table: NaN-poisoned padding/tails, fp32 reference). TunableOp only times candidates, so
this is the table's correctness gate."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tuned_table_solutions_correct():
    from gke_ray_train_amd.ops.gemm_tuning import check_tuned_table
    rows = check_tuned_table()
    assert rows, "no GEMM rows in the tuned table"
    bad = [(ln.split(",")[1], ln.split(",")[2], finite, rel) for ln, finite, rel, ok in rows if not ok]
    assert not bad, f"tuned solutions failing the poisoned-operand check: {bad}"


def test_poisoned_check_detects_reads_outside_operands():
    """The check itself: a correct default GEMM on a strided (padded) slice passes."""
    from gke_ray_train_amd.ops.gemm_tuning import check_gemm_row
    torch.cuda.tunable.enable(False)
    finite, rel = check_gemm_row("GemmTunableOp_BFloat16_TN", "tn_512_256_64_ld_64_192_768")
    assert finite and rel < 2e-2
