"""Adam beside the GEMM's LDS-DMA: bit-for-bit agreement of the riding bodies.

Round 5 found the float4 Adam riding in the split-K dW GEMM launch updating the low component of
16 consecutive lanes with denom = eps.  tools/probes/adam_ride_probe.hip pinned it down
(profiles/packed_fp32_lds_dma_r6.log): packed fp32 (v_pk_*_f32) results in a kernel whose waves
share a CU with LDS-DMA traffic (global_load_lds_dwordx4, the GEMM tiles' operand path) are wrong
now and then - in the same launch or in another kernel on another stream - while the same code
without packed fp32 never is.  gemm_bf16.hip and optim.hip are therefore compiled without packed
fp32 (_build.py FILE_FLAGS); here the float4 riding body, the scalar riding body (the executor's) and
the standalone Adam launch must agree bit for bit over repeated launches, each one from the same
state, with the GEMM tiles streaming beside the riding bodies.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nat():
    from dct_amd.ops._native import native

    return native()


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    M = N = 1024
    K, splits = 4096, 4
    n = 1 << 20
    dz = (torch.randn(K, M, device=dev) * 0.5).to(torch.bfloat16)
    x = (torch.randn(K, N, device=dev) * 0.5).to(torch.bfloat16)
    part = torch.empty(splits * M * N, device=dev)
    colsum = torch.zeros(M, device=dev)
    p0 = torch.randn(n, device=dev) * 0.05
    g = torch.randn(n, device=dev) * 1e-4          # tabular-scale gradients: v below 2^-32 (sqrtf's rescaled path)
    m0 = torch.randn(n, device=dev) * 1e-5
    v0 = torch.rand(n, device=dev) * 1e-12
    step = torch.tensor([3], dtype=torch.int32, device=dev)
    return dict(dz=dz, x=x, part=part, colsum=colsum, p0=p0, g=g, m0=m0, v0=v0, step=step, M=M, N=N, K=K,
                splits=splits, n=n)


def _run(s, mode):
    nat = _nat()
    p, m, v = s["p0"].clone(), s["m0"].clone(), s["v0"].clone()
    nat.adam_ride_check(mode, s["dz"].data_ptr(), s["x"].data_ptr(), s["part"].data_ptr(), s["colsum"].data_ptr(),
                        s["M"], s["N"], s["K"], s["splits"], p.data_ptr(), s["g"].data_ptr(), m.data_ptr(),
                        v.data_ptr(), s["n"], 1e-3, 0.9, 0.999, 1e-8, s["step"].data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return p, m, v


def test_riding_adam_bodies_match_standalone_bit_for_bit(setup):
    ref = _run(setup, 2)
    # sanity: the update is the torch.optim.Adam one (bias-corrected at t = 3)
    b1, b2, eps, lr, t = 0.9, 0.999, 1e-8, 1e-3, 3
    m = b1 * setup["m0"] + (1 - b1) * setup["g"]
    v = b2 * setup["v0"] + (1 - b2) * setup["g"] * setup["g"]
    want = setup["p0"] - lr / (1 - b1 ** t) * m / (v.sqrt() / (1 - b2 ** t) ** 0.5 + eps)
    # (the update itself to fp32 rounding: v reaches ~1e-20 here, where sqrt(v) / sqrt(1 - b2^t) is close to
    # eps and the two formulations' roundings of the bias corrections move the quotient by ~1e-5 of it)
    upd, want_upd = ref[0] - setup["p0"], want - setup["p0"]
    rel = (upd - want_upd).abs() / want_upd.abs().clamp_min(1e-12)
    assert float(rel.median()) < 1e-5 and float((upd - want_upd).abs().max()) < 1e-3 * float(want_upd.abs().max()), (
        float(rel.median()), float((upd - want_upd).abs().max()))
    for mode in (0, 1):  # scalar riding body, float4 riding body - beside the GEMM tiles' LDS-DMA
        for it in range(12):
            got = _run(setup, mode)
            for name, a, b in zip("pmv", got, ref):
                bad = (a.view(torch.int32) != b.view(torch.int32)).sum().item()
                assert bad == 0, f"mode {mode} launch {it}: {bad} elements of {name} differ from the standalone Adam"
