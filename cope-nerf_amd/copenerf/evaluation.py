"""Evaluation-time test-pose optimisation: the loop of
Evaluator.eval_optimization (eval.py:44-93) on the HIP renderer.

Per test view, a PoseRetriever initialised from the neighbouring training pose
(eval.py:46-51) is refined by Adam (eval_pose_lr, default.yaml:90) under a
MultiStepLR with milestones every num_epoch/5 epochs (eval.py:55): each batch
renders the view's sampled rays at the world time step with cos_anneal_ratio 1
(eval.py:65-72), takes compute_loss's L1 rgb term alone (eval.py:76-78), and
steps the pose optimiser; the epoch's mean L2 becomes a PSNR (model/common.py:601-609).
The optimised poses are saved to / loaded from `model_eval_pose.pt` (eval.py:57-93).

The gradient reaches the poses through the rays: the HIP backward returns
d loss / d rays_o, d rays_d (tests/test_gpu_raygrad.py, frozen-network case),
and autograd carries them through make_c2w.  The reference also accumulates
gradients into the (never stepped) network parameters; `freeze_networks=True`
(default) skips those weight gradients — the pose trajectory is the same, the
step does no parameter-gradient GEMMs.  Full-image rendering of the refined
views (eval.py:95-188) is copenerf.inference.render_image.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .rays import PoseRetriever


def mse2psnr(mse):
    """model/common.py:601-609."""
    mse = np.maximum(mse, 1e-10)
    return (20 * np.log10(1.0 / np.sqrt(mse))).astype(np.float32)


class EvalPoseOptimizer(object):
    """eval.py:44-93 for a Trainer (copenerf.trainer.Trainer, whose renderer is the HIP
    NeuSRenderer).  test_idx: the test views' image indices (i_test); init_c2w [n, 4, 4]:
    their starting poses (eval.py:47-48: the training pose of image idx - 1)."""

    def __init__(self, model, test_idx, init_c2w, world_time_step, cfg_eval, device=None, freeze_networks=True):
        self.model = model
        self.test_idx = [int(i) for i in test_idx]
        self.device = device if device is not None else init_c2w.device
        self.world_time_step = float(world_time_step)
        self.num_epoch = int(cfg_eval["eval_pose_epoch"])
        self.pose_retriever_test = PoseRetriever(len(self.test_idx), init_c2w=init_c2w).to(self.device)
        self.pose_optimizer = torch.optim.Adam(self.pose_retriever_test.parameters(), lr=cfg_eval["eval_pose_lr"])
        step = max(1, int(self.num_epoch / 5))  # range(0, E, int(E/5)); int(E/5) = 0 would raise there
        self.scheduler = torch.optim.lr_scheduler.MultiStepLR(self.pose_optimizer,
                                                              milestones=list(range(0, self.num_epoch, step)),
                                                              gamma=cfg_eval["eval_pose_scheduler_gamma"])
        self.freeze_networks = freeze_networks
        self.it = 0
        self.epoch_it = 0

    def _renderer_params(self):
        r = self.model.renderer
        return [p for p in r.parameters() if p.requires_grad]

    def step(self, batch):
        """One batch of eval.py:63-83; returns the batch's l2_mean (device scalar)."""
        image_idx = int(batch.get("img.idx"))
        world_mat = self.pose_retriever_test(self.test_idx.index(image_idx))
        (_, _, _, _, rays_o, rays_d, rays_d_norm, rgb_gt, _, _) = self.model.process_data(batch, world_mat, it=self.it,
                                                                                        epoch=self.epoch_it)
        near, far = self.model.near_far_from_sphere(rays_o, rays_d)
        t = torch.tensor([self.world_time_step], dtype=torch.float32, device=rays_o.device)
        out = self.model.renderer(rays_o, rays_d, rays_d_norm, t, near, far, background_rgb=None,
                                  cos_anneal_ratio=1.0, it=self.it, eval=False)
        loss_dict = self.model.compute_loss(batch, out["color_fine"], rgb_gt, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0,
                                            it=self.it, epoch=self.epoch_it)
        loss = loss_dict["loss_rgb"]
        self.pose_optimizer.zero_grad()
        loss.backward()
        self.pose_optimizer.step()
        return loss_dict["l2_mean"].detach()

    def run_epoch(self, loader):
        """One epoch over the test loader; returns the epoch's PSNR (eval.py:84-86)."""
        frozen = self._renderer_params() if self.freeze_networks else []
        for p in frozen:
            p.requires_grad_(False)
        try:
            l2 = [self.step(batch) for batch in loader]
        finally:
            for p in frozen:
                p.requires_grad_(True)
        self.scheduler.step()
        self.epoch_it += 1
        return mse2psnr(float(torch.stack(l2).mean().item())) if l2 else None

    def eval_optimization(self, loader, out_dir=None, on_epoch=None):
        """eval.py:57-93: optimise (and save) the test poses, or load them when
        <out_dir>/models/weights/model_eval_pose.pt exists."""
        path = None if out_dir is None else os.path.join(out_dir, "models", "weights", "model_eval_pose.pt")
        if path is not None and os.path.isfile(path):
            self.pose_retriever_test.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))
            return self.pose_retriever_test
        for epoch_i in range(self.num_epoch):
            psnr = self.run_epoch(loader)
            if on_epoch is not None:
                on_epoch(epoch_i, psnr)
        if path is not None:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            torch.save(self.pose_retriever_test.state_dict(), path)
        return self.pose_retriever_test
