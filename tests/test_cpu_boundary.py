"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/sgnn.h declares (no compute without a GPU), the Python
mirror has the reference's state_dict layout, and the product refuses CPU
tensors instead of falling back."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from tests.helpers import ROOT, golden, hparams, stats_of

HEADER = os.path.join(ROOT, "include", "sgnn.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(sgnn_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from sgnn_amd import _hip
    lib = _hip.load_library()
    syms = header_symbols()
    assert len(syms) >= 9, syms
    for s in syms:
        assert hasattr(lib, s), f"{s} missing from libsgnn_hip.so"
        assert s in _hip.SIGNATURES, f"{s} not bound in sgnn_amd/_hip.py"
    assert lib.sgnn_version().decode().startswith("sgnn")


def test_header_constants_match_python_mirror():
    """The one-launch step's counter buffer size / error-word index (include/sgnn.h) as the
    Python workspace allocates and reads them (the kernel's static_assert pins the C side)."""
    from sgnn_amd import _hip
    src = open(HEADER).read()
    words = int(re.search(r"#define SGNN_STEP_FLAG_WORDS (\d+)", src).group(1))
    err = int(re.search(r"#define SGNN_STEP_FLAG_ERR (\d+)", src).group(1))
    assert (words, err) == (_hip.STEP_FLAG_WORDS, _hip.STEP_FLAG_ERR)
    assert 256 * 16 <= err < words   # 256 counters 64 B apart, then the error word
    abi = int(re.search(r"#define SGNN_ABI_VERSION (\d+)", src).group(1))
    lib = _hip.load_library()
    assert abi == _hip.ABI_VERSION == lib.sgnn_abi_version()
    assert lib.sgnn_step_flag_words() == words


def test_step_workspace_struct_size_leads_the_struct():
    """ABI guard (include/sgnn.h): sgnn_step_ws starts with struct_size, which the Python mirror fills
    with its own size; a caller built against another header revision is refused (CPU-side: the
    check runs before any device work, so a wrong size returns SGNN_ERR_INVALID without a GPU)."""
    from sgnn_amd import _hip
    assert _hip.SgnnStepWs._fields_[0] == ("struct_size", ctypes.c_int64)
    ws = _hip.SgnnStepWs(struct_size=ctypes.sizeof(_hip.SgnnStepWs) - 8)
    lib = _hip.load_library()
    assert lib.sgnn_step_check(ctypes.byref(ws), None) == _hip.SGNN_ERR_INVALID
    assert "struct_size" in lib.sgnn_last_error().decode()


def test_host_only_size_queries():
    from sgnn_amd import _hip
    lib = _hip.load_library()
    assert lib.sgnn_radius_workspace_bytes(50000, 20, 1) > 50000 * 20 * 4
    assert lib.sgnn_edge_latent_floats(33, 64) == 64 * 64  # 2 tiles of 32 edges


def test_state_dict_layout_and_init_match_reference():
    """Same module tree + construction order => torch.manual_seed(0) gives the
    reference's exact initial weights (golden 'w/' arrays were made that way)."""
    from sgnn_amd.learned_simulator import LearnedSimulator
    z = golden("tiny2d_r06")
    hp = hparams(z)
    torch.manual_seed(0)
    d, T, H = hp["dim"], hp["T"], hp["H"]
    sim = LearnedSimulator(d, (T - 1) * d + 1, d + 1, H, hp["L"], 1, H, hp["R"], stats_of(z), 1, 9)
    sd = sim.state_dict()
    ref_keys = sorted(k[2:] for k in z.files if k.startswith("w/"))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:
        np.testing.assert_array_equal(sd[k].numpy(), z["w/" + k], err_msg=k)


def test_product_refuses_cpu_tensors():
    from tests.helpers import product_sim
    z = golden("tiny2d_r06")
    sim = product_sim(z, device="cpu")
    pos = torch.from_numpy(z["positions"][:, :11])
    with pytest.raises(ValueError, match="GPU"):
        sim.predict_positions(pos, [pos.shape[0]], torch.zeros(pos.shape[0], dtype=torch.long))


def test_reference_input_validation():
    from tests.helpers import product_sim
    sim = product_sim(golden("tiny2d_r06"), device="cpu")
    with pytest.raises(ValueError, match="3 dimensions"):
        sim.predict_positions(torch.zeros(5, 2), [5], torch.zeros(5, dtype=torch.long))
    with pytest.raises(ValueError, match="at least 2 timesteps"):
        sim.predict_positions(torch.zeros(5, 1, 2), [5], torch.zeros(5, dtype=torch.long))
    with pytest.raises(ValueError, match="2D positions"):
        sim._compute_graph_connectivity(torch.zeros(5, 1, 2), [5], 0.6)


@pytest.mark.parametrize("case,seed", [("ms2d_s3", 3), ("ms3d_h128", 4)])
def test_multi_scale_state_dict_and_init_match_reference(case, seed):
    """MultiScaleSimulator: same keys, same construction order => same init."""
    from sgnn_amd.multi_scale import MultiScaleSimulator
    z = golden(case)
    hp = hparams(z)
    d, T, H = hp["dim"], hp["T"], hp["H"]
    torch.manual_seed(seed)
    nnode_in = (T - 1) * d + 1 + (hp["emb"] if hp["ntypes"] > 1 else 0)
    sim = MultiScaleSimulator(d, nnode_in, d + 1, H, H, hp["L"], hp["nmlp"], stats_of(z), hp["ntypes"],
                              hp["emb"], hp["num_scales"], hp["window"], hp["mult"])
    sd = sim.state_dict()
    ref_keys = sorted(k[2:] for k in z.files if k.startswith("w/"))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:
        np.testing.assert_array_equal(sd[k].numpy(), z["w/" + k], err_msg=k)


def test_multi_scale_validation():
    from sgnn_amd.multi_scale import MultiScaleConfig, MultiScaleSimulator
    with pytest.raises(ValueError, match="num_scales"):
        MultiScaleConfig(num_scales=1)
    z = golden("ms2d_s3")
    hp = hparams(z)
    sim = MultiScaleSimulator(2, 11, 3, 64, 64, 1, 2, stats_of(z), 1, 9, 3, 2, 2.0)
    with pytest.raises(ValueError, match="Static graph data not set"):
        sim._validate_static_graph()
    sim.set_static_graph({"graph_hierarchy": {}})
    with pytest.raises(ValueError, match="Missing required graph data key"):
        sim._validate_static_graph()
    with pytest.raises(ValueError, match="GPU"):
        sim.predict_positions(torch.zeros(5, 6, 2), [5], None)


def test_every_module_compiles():
    """Every Python source of the package, the bench and the tools parses (a
    syntax error in a module only the GPU path imports must fail here, on CPU)."""
    import pathlib
    import py_compile
    root = pathlib.Path(__file__).resolve().parents[1]
    files = sorted(root.glob("sgnn_amd/**/*.py")) + [root / "bench.py", root / "__graft_entry__.py"] + \
        sorted(root.glob("tools/*.py")) + sorted(root.glob("oracle/*.py"))
    for f in files:
        py_compile.compile(str(f), doraise=True)
