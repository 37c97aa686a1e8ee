"""Training driver -- the reference's ``train_kitti.py`` (NOFSystem + Lightning Trainer.fit) without Lightning.

Same command line (nof.nof_utils.get_opts), same model/loss/optimizer/scheduler construction and the same
training / validation step arithmetic (train_kitti.py:20-245); what Lightning did around it is written out here:

  * data: the ray tables are built on the GPU and stay in HBM (nof.dataset.kitti_dataload); each epoch walks a
    device ``randperm`` in batches of ``batch_size`` rays (DataLoader(shuffle=True), last batch kept) -- no worker
    processes, no host->device copy per batch;
  * step: zero_grad, training_step, loss.backward() through the HIP backward kernels, optimizer.step();
    MultiStepLR([5, 120, 256], decay_gamma) stepped once per epoch (Lightning's default interval);
  * validation: the full val set before training (num_sanity_val_steps=-1) and after every epoch, batches of
    ``batch_size_val``, metrics averaged over batches;
  * checkpoints: Lightning layout {'state_dict': {'nof_coarse.*', 'nof_fine.*'}} -- last.ckpt every epoch,
    best.ckpt on the lowest train/loss -- loadable by the reference's load_ckpt;
  * data parallel (one process per GPU, ``torchrun``): every rank takes its slice of each global batch of
    ``batch_size * world`` rays (DistributedSampler semantics), gradients are averaged with one all_reduce of a
    flat bucket over RCCL (nof.blocks.allreduce_grads); each chunk is normalised by its own batch statistics on
    its rank (no sync_batchnorm, as Lightning's DDP), while the BatchNorm RUNNING statistics are made
    rank-independent (nof.bn_sync: every rank's chunk statistics replayed in global chunk order), so every rank's
    checkpoint is the same.

Usage (PC-NeRF KITTI-00 1151-1200, shells/pretraining/KITTI00_pcnerf_train.bash's options):
    python pc-nerf_amd/train_kitti.py --datasettype kitti_dataload --root_dir <pcd dir> --pose_path poses.txt \\
        --data_start 1150 --data_end 1200 --re_loaddata 1 --result_path logs/kitti00 --N_samples 768 ...
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from torch.optim.lr_scheduler import MultiStepLR  # noqa: E402

from nof.blocks import allreduce_grads, shard_batch  # noqa: E402
from nof.bn_sync import BnSync  # noqa: E402
from nof.criteria import child_range_loss, nof_loss  # noqa: E402
from nof.criteria.metrics import abs_error, acc_thres, eval_points  # noqa: E402
from nof.dataset import nof_dataset  # noqa: E402
from nof.io import load_ckpt, save_ckpt  # noqa: E402
from nof.networks import Embedding, NOF_coarse, NOF_fine  # noqa: E402
from nof.nof_utils import decode_batch, get_learning_rate, get_opts, get_optimizer  # noqa: E402
from nof.render import render_rays_train, render_rays_val  # noqa: E402

PLOT_KEYS = ('', '_range', '_range_fine', '_child_free', '_child_free_fine', '_child_depth', '_child_depth_fine')


class NOFSystem:
    """train_kitti.py:20-245 (NOFSystem(LightningModule)) as a plain object."""

    def __init__(self, hparams, train_dataset=None, val_dataset=None):
        self.hparams = hparams
        self.device = torch.device(hparams.device)
        self.embedding_position = Embedding(in_channels=3, N_freq=hparams.L_pos)
        cin = 3 + 3 * hparams.L_pos * 2
        self.nof_coarse = NOF_coarse(feature_size=hparams.feature_size, in_channels_xy=cin,
                                     use_skip=hparams.use_skip).to(self.device)
        self.nof_fine = NOF_fine(feature_size=hparams.feature_size, in_channels_xy=cin,
                                 use_skip=hparams.use_skip).to(self.device)
        if hparams.ckpt_path:
            load_ckpt(self.nof_coarse, hparams.ckpt_path, model_name='nof_coarse')
            load_ckpt(self.nof_fine, hparams.ckpt_path, model_name='nof_fine')
        self.loss = nof_loss[hparams.loss_type]()
        self.train_dataset, self.val_dataset = train_dataset, val_dataset
        self.plots = {k: [] for k in ('x',) + PLOT_KEYS}

    # ------------------------------------------------------------------ data (train_kitti.py:46-83)
    def prepare_data(self):
        h = self.hparams
        if self.train_dataset is not None:
            return
        common = dict(root_dir=h.root_dir, data_start=h.data_start, data_end=h.data_end,
                      cloud_size_val=h.cloud_size_val, range_delete_x=h.range_delete_x,
                      range_delete_y=h.range_delete_y, range_delete_z=h.range_delete_z,
                      sub_nerf_test_num=h.sub_nerf_test_num, pose_path=h.pose_path, subnerf_path=h.subnerf_path,
                      surface_expand=h.surface_expand, re_loaddata=h.re_loaddata, result_path=h.result_path,
                      device=self.device, sparsity=h.frame_sparsity)
        if h.datasettype == "kitti_dataload":
            kwargs = dict(common, parentnerf_path=h.parentnerf_path, interest_x=h.interest_x,
                          interest_y=h.interest_y, over_height=h.over_height, over_low=h.over_low)
        elif h.datasettype == "maicity_dataload":
            kwargs = dict(common, nerf_length_min=h.nerf_length_min, nerf_length_max=h.nerf_length_max,
                          nerf_width_min=h.nerf_width_min, nerf_width_max=h.nerf_width_max,
                          nerf_height_min=h.nerf_height_min, nerf_height_max=h.nerf_height_max)
        else:
            raise NotImplementedError(f"datasettype {h.datasettype!r}: kitti_dataload or maicity_dataload")
        ds = nof_dataset[h.datasettype]
        self.train_dataset = ds(split='train', **kwargs)
        self.val_dataset = ds(split='val', **kwargs)

    # ------------------------------------------------------------------ model (train_kitti.py:85-115)
    def forward(self, rays, isval):
        h = self.hparams
        common = dict(model=self.nof_coarse, model_fine=self.nof_fine, embedding_xy=self.embedding_position,
                      rays=rays, N_samples=h.N_samples, N_importance=h.N_importance, use_disp=h.use_disp,
                      perturb=h.perturb, noise_std=h.noise_std, chunk=h.chunk, isval=isval,
                      sub_nerf_test_num=h.sub_nerf_test_num)
        if not isval:
            return render_rays_train(**common, issegmentated=h.use_segmentated_sample,
                                     childnerf_ratio=h.segmentated_child_nerf_ratio,
                                     use_child_nerf_divide=h.use_child_nerf_divide,
                                     use_child_nerf_loss=h.use_child_nerf_loss)
        return render_rays_val(**common)

    def parameters(self):
        return list(self.nof_coarse.parameters()) + list(self.nof_fine.parameters())

    def configure_optimizers(self):
        self.optimizer = get_optimizer(self.hparams, self.parameters())
        self.scheduler = MultiStepLR(self.optimizer, milestones=[5, 120, 256], gamma=self.hparams.decay_gamma)
        return self.optimizer, self.scheduler

    # ------------------------------------------------------------------ steps (train_kitti.py:117-245)
    def range_losses(self, rays, pred, pred_fine, gt):
        h = self.hparams
        if h.use_child_nerf_divide == 1:    # train_kitti.py:125-142, one kernel pair per term
            return (child_range_loss(pred, gt, rays, h.sub_nerf_test_num, h.lambda_loss),
                    child_range_loss(pred_fine, gt, rays, h.sub_nerf_test_num, h.lambda_loss_fine))
        # train_kitti.py:144-146 (the reference scales the fine term by lambda_loss too)
        return (1e-1 * h.lambda_loss * self.loss(1e1 * pred, 1e1 * gt),
                1e-1 * h.lambda_loss * self.loss(1e1 * pred_fine, 1e1 * gt))

    def training_step(self, batch, batch_idx):
        h = self.hparams
        rays, gt = decode_batch(batch)
        res = self.forward(rays, False)
        pred, pred_fine = res['depth'], res['depth_fine']
        loss_range, loss_range_fine = self.range_losses(rays, pred, pred_fine, gt)
        cf, cff = res['child_free_loss'], res['child_free_loss_fine']
        cd, cdf = res['child_depth_loss'], res['child_depth_loss_fine']
        dev = pred.device
        cf, cff, cd, cdf = (t.to(dev) for t in (cf, cff, cd, cdf))   # disabled child losses are CPU zeros
        loss = (loss_range + loss_range_fine + h.lambda_child_free_loss * cff + h.lambda_child_free_loss * cf
                + h.lambda_child_depth_loss * cdf + h.lambda_child_depth_loss * cd)
        with torch.no_grad():
            logs = {'train/loss': loss.detach(), 'train/avg_error': abs_error(pred, gt), 'train/acc_thres': acc_thres(pred, gt),
                    'lr': get_learning_rate(self.optimizer)}
            self._record_plot(batch_idx, loss, loss_range, loss_range_fine, h.lambda_child_free_loss * cf,
                              h.lambda_child_free_loss * cff, h.lambda_child_depth_loss * cd,
                              h.lambda_child_depth_loss * cdf)
        return loss, logs

    def _record_plot(self, batch_idx, *terms):
        """train_kitti.py:163-196: every 5th batch (after the first 20 of epoch 0) the loss terms are appended to
        the ploty arrays, saved with np.save when the paths are given."""
        h = self.hparams
        if not ((h.current_epoch != 0) or (batch_idx >= 20)) or batch_idx % 5 != 0:
            return
        if h.current_epoch == 0:
            h.current_epoch += 1
            self.plots['x'].append(1)
        else:
            self.plots['x'].append(len(self.plots['x']) + 1)
        for k, t in zip(PLOT_KEYS, terms):
            self.plots[k].append(np.asarray(t.detach().float().cpu().numpy()))
            path = getattr(h, 'saveploty_path' + k, None)
            if path:
                os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
                np.save(path, arr=self.plots[k])

    @torch.no_grad()
    def validation_step(self, batch, batch_idx):
        h = self.hparams
        rays, gt = decode_batch(batch)
        rays, gt = rays.squeeze(), gt.squeeze()
        res = self.forward(rays, True)
        pred = res['depth_fine']
        o, d = rays[:, :3], rays[:, 3:6]
        cd, fscore = eval_points(o + d * pred.unsqueeze(-1), o + d * gt.unsqueeze(-1))
        if h.use_child_nerf_divide == 1:    # train_kitti.py:213-236: mean over the children present
            sub = rays[:, 9]
            k = torch.floor(sub - 0.5).to(torch.int64)
            ok = (k >= 0) & (k < h.sub_nerf_test_num) & (sub > k + 0.5) & (sub < k + 1.5)
            present = torch.unique(k[ok])
            losses, errs, accs = [], [], []
            for c in present.tolist():
                m = ok & (k == c)
                losses.append(self.loss(pred[m], gt[m]))
                errs.append(abs_error(pred[m], gt[m]))
                accs.append(acc_thres(pred[m], gt[m]))
            n = max(len(losses), 1)
            loss, err, acc = sum(losses) / n, sum(errs) / n, sum(accs) / n
        else:
            loss, err, acc = self.loss(pred, gt), abs_error(pred, gt), acc_thres(pred, gt)
        return {'val/loss': float(loss), 'val/avg_error': float(err), 'val/acc_thres': float(acc), 'val/cd': cd,
                'val/fscore': fscore}


def _log(fh, rec):
    if fh is not None:
        fh.write(json.dumps({k: (float(v) if torch.is_tensor(v) else v) for k, v in rec.items()}) + "\n")
        fh.flush()


def validate(system, fh=None, epoch=-1):
    h, ds = system.hparams, system.val_dataset
    if ds is None or len(ds) == 0:
        return {}
    system.nof_coarse.eval()
    system.nof_fine.eval()
    recs = []
    for b, s in enumerate(range(0, len(ds), h.batch_size_val)):
        recs.append(system.validation_step(ds[torch.arange(s, min(s + h.batch_size_val, len(ds)))], b))
    out = {k: float(np.mean([r[k] for r in recs])) for k in recs[0]}
    _log(fh, {"epoch": epoch, **out})
    return out


def fit(system, max_steps=0, log_path=None, ckpt_dir=None):
    """Trainer.fit (train_kitti.py:286-299) for one process, or one rank of a data-parallel job."""
    import torch.distributed as dist
    h = system.hparams
    ddp = dist.is_available() and dist.is_initialized()
    rank, world = (dist.get_rank(), dist.get_world_size()) if ddp else (0, 1)
    bns = BnSync() if ddp else None
    system.prepare_data()
    opt, sched = system.configure_optimizers()
    params = system.parameters()
    fh = open(log_path, "a") if (log_path and rank == 0) else None
    best = float("inf")
    val = validate(system, fh, -1) if rank == 0 else {}          # num_sanity_val_steps=-1
    n = len(system.train_dataset)
    gen = torch.Generator(device=system.device).manual_seed(int(h.seed or 0))
    step = 0
    t0 = time.perf_counter()
    for epoch in range(h.num_epochs):
        system.nof_coarse.train()
        system.nof_fine.train()
        perm = torch.randperm(n, device=system.device, generator=gen)   # same order on every rank (same seed)
        gb = h.batch_size * world
        ep_loss = []
        for b, s in enumerate(range(0, n, gb)):
            glob = perm[s:s + gb]
            if glob.numel() < world:   # a rank's shard would be empty: every rank skips it (the collectives below)
                continue
            idx = shard_batch(glob, rank, world)
            opt.zero_grad(set_to_none=True)
            if ddp:
                with bns.record():
                    loss, logs = system.training_step(system.train_dataset[idx], b)
            else:
                loss, logs = system.training_step(system.train_dataset[idx], b)
            loss.sum().backward()
            if ddp:
                allreduce_grads(params)
                bns.sync()
            opt.step()
            step += 1
            ep_loss.append(loss.detach())
            if fh is not None and (b % 10 == 0):
                _log(fh, {"epoch": epoch, "step": step, **logs})
            if max_steps and step >= max_steps:
                break
        sched.step()
        if rank == 0 and ep_loss:
            mean_loss = float(torch.stack([l.reshape(()) for l in ep_loss]).mean())
            if ckpt_dir:
                os.makedirs(ckpt_dir, exist_ok=True)
                save_ckpt(os.path.join(ckpt_dir, "last.ckpt"), nof_coarse=system.nof_coarse, nof_fine=system.nof_fine)
                if mean_loss < best:
                    best = mean_loss
                    save_ckpt(os.path.join(ckpt_dir, "best.ckpt"), nof_coarse=system.nof_coarse,
                              nof_fine=system.nof_fine)
            val = validate(system, fh, epoch)
        if max_steps and step >= max_steps:
            break
    torch.cuda.synchronize(system.device) if system.device.type == "cuda" else None
    if fh is not None:
        fh.close()
    return {"steps": step, "seconds": time.perf_counter() - t0, "val": val}


def main(argv=None):
    h = get_opts(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        h.device = f"cuda:{local}"
    if h.seed:
        torch.manual_seed(h.seed)
        np.random.seed(h.seed)
    system = NOFSystem(h)
    out_dir = os.path.join("logs", h.exp_name) if not h.result_path else h.result_path
    res = fit(system, max_steps=h.max_steps, log_path=h.log_path,
              ckpt_dir=os.path.join(out_dir, "checkpoints"))
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
