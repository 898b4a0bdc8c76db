"""CheckpointIO: drop-in for model/checkpoints.py:9-131 (train.py:94-113 saves and
resumes through it).  Same directory layout (<dir>/models/weights[_<epoch>]/<file>),
same dict format ({module name: state_dict} plus scalars), so checkpoints move
between the reference and this build in both directions: tests/test_checkpoint_layout.py
loads a checkpoint the reference's own CheckpointIO wrote (DataParallel renderer with
`module.`-prefixed keys incl. the motion network, both Adam optimizers, epoch_it / it /
depth_range; train.py:54, 94, 158-167) strictly, and checks that what this class saves
has the same keys, shapes, dtypes and optimizer-state layout.  Loading uses
torch.load(weights_only=True): a checkpoint is data, never code.  URL loading
(model_zoo, checkpoints.py:102-112) is not offered: no network here."""
from __future__ import annotations

import datetime
import os
import shutil

import torch


class CheckpointIO(object):
    def __init__(self, checkpoint_dir="./chkpts", **kwargs):
        self.module_dict = kwargs
        self.checkpoint_dir = checkpoint_dir
        os.makedirs(checkpoint_dir, exist_ok=True)

    def register_modules(self, **kwargs):
        self.module_dict.update(kwargs)

    def save(self, filename, lastest_checkpoint, **kwargs):
        """checkpoints.py:29-46 (the reference's argument name `lastest_checkpoint` kept)."""
        sub = "weights" if lastest_checkpoint else f'weights_{kwargs["epoch_it"]}'
        save_dir = os.path.join(self.checkpoint_dir, "models", sub)
        os.makedirs(save_dir, exist_ok=True)
        if not os.path.isabs(filename):
            filename = os.path.join(save_dir, filename)
        outdict = dict(kwargs)
        for k, v in self.module_dict.items():
            outdict[k] = v.state_dict()
        torch.save(outdict, filename)

    def backup_model_best(self, filename, **kwargs):
        if not os.path.isabs(filename):
            filename = os.path.join(self.checkpoint_dir, filename)
        if os.path.exists(filename):
            backup_dir = os.path.join(self.checkpoint_dir, "backup_model_best")
            os.makedirs(backup_dir, exist_ok=True)
            shutil.copy(filename, os.path.join(backup_dir, "%s.pt" % datetime.datetime.now().timestamp()))

    def load(self, filename, device=None, load_epoch=None, load_model_only=False):
        """checkpoints.py:58-74."""
        if load_epoch is not None:
            filename = filename.replace("/weights/", f"/weights_{load_epoch}/")
        return self.load_file(filename, device, load_model_only)

    def load_file(self, filename, device=None, load_model_only=False):
        if not os.path.exists(filename):
            raise FileExistsError(filename)  # the reference's (sic) exception type
        state_dict = torch.load(filename, map_location=device, weights_only=True)
        if load_model_only:
            state_dict = {"model": state_dict["model"]}
        return self.parse_state_dict(state_dict)

    def parse_state_dict(self, state_dict):
        """checkpoints.py:114-131: strict load of every registered module; the rest are scalars."""
        for k, v in self.module_dict.items():
            if k in state_dict:
                v.load_state_dict(state_dict[k])
            else:
                print("Warning: Could not find %s in checkpoint!" % k)
        return {k: v for k, v in state_dict.items() if k not in self.module_dict}
