"""The checkpoint train.py writes against fixtures the reference
wrote itself (tests/golden/make_golden.py, checkpoint_case):
  * the state-dict keys and shapes of DataParallel(NeuSRenderer(None, sdf, dev, col,
    motion)) at the default.yaml widths (train.py:47-54: every key `module.`-prefixed);
  * a checkpoint file saved by the reference's model/checkpoints.py CheckpointIO with
    model = that DataParallel renderer, optimizer / motion_optimizer = the two Adam
    optimizers after a step (train.py:57-59, 94), and epoch_it / it / depth_range
    (train.py:158-167): this build's CheckpointIO loads it strictly, and what it saves has
    the same structure (keys, shapes, dtypes, optimizer state layout).  CPU only."""
import json
import os
import tempfile

import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _build(width=None):
    from copenerf.fields import RenderingNetwork, SDFNetwork, SingleVarianceNetwork
    from copenerf.motion import MotionNetwork
    from copenerf.renderer import NeuSRenderer
    from copenerf.train_step import COL_CFG, MOTION_CFG, REN_CFG, SDF_CFG
    torch.manual_seed(700)
    w = {} if width is None else {"d_hidden": width}
    sdf = SDFNetwork(**dict(SDF_CFG, **w))
    col = RenderingNetwork(**dict(COL_CFG, **w, **({} if width is None else {"d_feature": width})))
    dev = SingleVarianceNetwork(0.3)
    motion = MotionNetwork(**dict(MOTION_CFG, **w))
    dp = torch.nn.DataParallel(NeuSRenderer(None, sdf, dev, col, motion, **REN_CFG))
    opt = torch.optim.Adam(list(sdf.parameters()) + list(dev.parameters()) + list(col.parameters()), lr=1e-3)
    mopt = torch.optim.Adam(motion.parameters(), lr=5e-4)
    return dp, opt, mopt


def test_dataparallel_renderer_state_dict_keys_match_reference():
    ref = json.load(open(os.path.join(GOLD, "state_keys.json")))["keys"]
    dp, _, _ = _build()
    ours = {k: list(v.shape) for k, v in dp.state_dict().items()}
    assert ours == ref


def _structure(sd):
    """Keys, shapes and dtypes of a checkpoint dict (optimizer states included)."""
    out = {}
    for k, v in sd.items():
        if k in ("optimizer", "motion_optimizer"):
            out[k] = {"groups": [sorted(g) for g in v["param_groups"]],
                      "state": {i: {n: (list(t.shape), str(t.dtype)) for n, t in s.items()} for i, s in v["state"].items()}}
        elif isinstance(v, dict):
            out[k] = {n: (list(t.shape), str(t.dtype)) for n, t in v.items()}
        else:
            out[k] = type(v).__name__
    return out


def test_reference_checkpoint_loads_strictly_and_saves_the_same_layout():
    from copenerf.checkpoints import CheckpointIO
    path = os.path.join(GOLD, "ref_checkpoint.pt")
    ref = torch.load(path, map_location="cpu", weights_only=True)
    dp, opt, mopt = _build(64)
    with tempfile.TemporaryDirectory() as d:
        io = CheckpointIO(d, model=dp, optimizer=opt, motion_optimizer=mopt)
        scalars = io.load_file(path)
        assert scalars == {"epoch_it": 12, "it": 3456, "depth_range": [0.01, 5.0]}
        for k, v in dp.state_dict().items():
            assert torch.equal(v, ref["model"][k]), k
        for o, name in ((opt, "optimizer"), (mopt, "motion_optimizer")):
            st = o.state_dict()["state"]
            assert st.keys() == ref[name]["state"].keys()
            for i, s in st.items():
                for n, t in s.items():
                    assert torch.equal(t, ref[name]["state"][i][n]), (name, i, n)
        io.save("model.pt", lastest_checkpoint=True, epoch_it=12, it=3456, depth_range=[0.01, 5.0])
        ours = torch.load(os.path.join(d, "models", "weights", "model.pt"), map_location="cpu", weights_only=True)
        assert _structure(ours) == _structure(ref)
        # and what this build saved loads back into a fresh build, value for value
        dp2, opt2, mopt2 = _build(64)
        io2 = CheckpointIO(d, model=dp2, optimizer=opt2, motion_optimizer=mopt2)
        io2.load(os.path.join(d, "models", "weights", "model.pt"))
        for (k, a), b in zip(dp.state_dict().items(), dp2.state_dict().values()):
            assert torch.equal(a, b), k
