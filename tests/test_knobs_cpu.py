"""The native launchers' DCT_* knobs (csrc/knobs.h): read once into one struct at plan / bind time
(reload_knobs), never on a launch path - pinned on CPU through the extension's introspection hook.
Skips where the extension cannot be imported (no HIP runtime)."""
import pytest

from dct_amd.ops import _native


@pytest.fixture
def nat():
    if not _native.available():
        pytest.skip("native extension not importable here")
    n = _native.native()
    yield n
    n.reload_knobs()  # torn down after monkeypatch (requested first): back to the real environment


def test_knobs_defaults_and_reload(nat, monkeypatch):
    for k in ("DCT_MLP_BLOCK", "DCT_FUSED_HEAD", "DCT_REDUCER_INLINE", "DCT_REDUCER_STANDIN_US", "DCT_DW_INTO_ADAM"):
        monkeypatch.delenv(k, raising=False)
    nat.reload_knobs()
    d = nat.knobs()
    assert d["mlp_block"] == -1 and d["fused_head"] == 1 and d["dw_into_adam"] == 1
    assert d["reducer_inline"] == -2 and d["reducer_standin_us"] == 0 and d["reducer_standin_wgs"] == 16
    monkeypatch.setenv("DCT_MLP_BLOCK", "3")
    monkeypatch.setenv("DCT_FUSED_HEAD", "0")
    monkeypatch.setenv("DCT_REDUCER_STANDIN_US", "60")
    # the environment alone changes nothing: the struct is re-read only at plan / bind time
    assert nat.knobs()["mlp_block"] == -1
    nat.reload_knobs()
    d = nat.knobs()
    assert d["mlp_block"] == 3 and d["fused_head"] == 0 and d["reducer_standin_us"] == 60
    monkeypatch.setenv("DCT_MLP_BLOCK", "0")
    monkeypatch.setenv("DCT_REDUCER_INLINE", "7")  # out of range: back to auto
    nat.reload_knobs()
    assert nat.knobs()["mlp_block"] == 0 and nat.knobs()["reducer_inline"] == -2


def test_knob_count_stays_small():
    """measured-and-rejected variants are deleted with their knobs.  Every DCT_* name the
    package, bench.py and jobs/ read (config surface, orchestration, tests' A/B hooks included)."""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = set()
    for base in ("distributed-continuous-training-with-airflow-pytorch-distributed-ddp-_amd", "jobs"):
        for dp, _, fs in os.walk(os.path.join(root, base)):
            for f in fs:
                if f.endswith((".py", ".cpp", ".h", ".hip")):
                    names |= set(re.findall(r"DCT_[A-Z0-9_]+", open(os.path.join(dp, f)).read()))
    names |= set(re.findall(r"DCT_[A-Z0-9_]+", open(os.path.join(root, "bench.py")).read()))
    assert len(names) <= 60, sorted(names)


def test_mlp_plan_reloads_knobs(nat, monkeypatch):
    """FusedMLPKernel's native plan re-reads the knobs when it is built."""
    monkeypatch.setenv("DCT_MLP_KERNEL", "lds")
    nat.reload_knobs()
    assert nat.knobs()["mlp_force_lds"] == 1
    monkeypatch.setenv("DCT_MLP_KERNEL", "auto")
    nat.MlpPlan([5, 64, 2], 4)
    assert nat.knobs()["mlp_force_lds"] == 0


def test_block_choice_is_a_plan_time_copy(nat, monkeypatch):
    """the 3x128 launch path (dct_mlp_train, mlp_block3_ok) reads DCT_MLP_BLOCK from the
    plan's own copy, stamped when the MlpPlan is built - a later reload of the process-wide knobs does not
    change an existing plan's launches."""
    monkeypatch.setenv("DCT_MLP_BLOCK", "3")
    plan = nat.MlpPlan([5, 128, 128, 2], 4)
    assert plan.mlp_block == 3
    monkeypatch.setenv("DCT_MLP_BLOCK", "0")
    nat.reload_knobs()
    assert nat.knobs()["mlp_block"] == 0 and plan.mlp_block == 3
    assert nat.MlpPlan([5, 128, 128, 2], 4).mlp_block == 0
    monkeypatch.delenv("DCT_MLP_BLOCK")
    assert nat.MlpPlan([5, 128, 128, 2], 4).mlp_block == -1
