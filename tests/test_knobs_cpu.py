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
    for k in ("DCT_GEMM_STAGES", "DCT_MLP_BLOCK", "DCT_TT_HEAD_SPB", "DCT_FUSED_HEAD", "DCT_REDUCER_INLINE"):
        monkeypatch.delenv(k, raising=False)
    nat.reload_knobs()
    d = nat.knobs()
    assert d["gemm_stages"] == 0 and d["mlp_block"] == -1 and d["tt_head_spb"] == 4
    assert d["fused_head"] == 1 and d["reducer_inline"] == -2 and d["reducer_standin_us"] == 0 and d["gemm_bm64_nk"] == 4
    monkeypatch.setenv("DCT_GEMM_STAGES", "4")
    monkeypatch.setenv("DCT_MLP_BLOCK", "3")
    monkeypatch.setenv("DCT_TT_HEAD_SPB", "16")
    monkeypatch.setenv("DCT_FUSED_HEAD", "0")
    # the environment alone changes nothing: the struct is re-read only at plan / bind time
    assert nat.knobs()["gemm_stages"] == 0
    nat.reload_knobs()
    d = nat.knobs()
    assert d["gemm_stages"] == 4 and d["mlp_block"] == 3 and d["tt_head_spb"] == 16 and d["fused_head"] == 0
    monkeypatch.setenv("DCT_MLP_BLOCK", "0")
    monkeypatch.setenv("DCT_TT_HEAD_SPB", "7")  # only 4 or 16
    nat.reload_knobs()
    assert nat.knobs()["mlp_block"] == 0 and nat.knobs()["tt_head_spb"] == 4


def test_mlp_plan_reloads_knobs(nat, monkeypatch):
    """FusedMLPKernel's native plan re-reads the knobs when it is built."""
    monkeypatch.setenv("DCT_MLP_KERNEL", "lds")
    nat.reload_knobs()
    assert nat.knobs()["mlp_force_lds"] == 1
    monkeypatch.setenv("DCT_MLP_KERNEL", "auto")
    nat.MlpPlan([5, 64, 2], 4)
    assert nat.knobs()["mlp_force_lds"] == 0
