"""Driver utilities -- drop-in for ``nof/nof_utils.py``: the command line of the training / evaluation drivers
(``get_opts``, nof_utils.py:8-152, same option names and defaults), the optimizer factory (:158-173), the batch
decoder (:202-210) and checkpoint loading (:176-199, via nof.io with ``weights_only=True``)."""
from __future__ import annotations

import argparse

from torch.optim import SGD, Adam

from .io import extract_model_state_dict, load_ckpt  # noqa: F401  (re-exported like the reference)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    a = p.add_argument
    # data (nof_utils.py:11-62)
    a('--result_path', type=str, default=None)
    a('--re_loaddata', type=int, default=0)
    a('--datasettype', type=str, default='kitti_sequence00_repeat')
    a('--root_dir', type=str, default='/media/bit/T7/dataset/kitti/dataset/sequences/00/pcd')
    a('--pose_path', type=str, default='/media/bit/T7/dataset/kitti/dataset/sequences/00/poses.txt')
    a('--data_start', type=int, default=1)
    a('--data_end', type=int, default=2)
    a('--parentnerf_path', type=str, default=None)
    a('--subnerf_path', type=str, default=None)
    a('--sub_nerf_test_num', type=int, default=3)
    a('--range_delete_x', type=float, default=2)
    a('--range_delete_y', type=float, default=1)
    a('--range_delete_z', type=float, default=0.5)
    a('--over_height', type=float, default=0.168)
    a('--over_low', type=float, default=-2.0)
    a('--interest_x', type=float, default=12)
    a('--interest_y', type=float, default=10)
    a('--cloud_size_val', type=int, default=128)
    a('--surface_expand', type=float, default=0.5)
    a('--nerf_length_min', type=float, default=-4.5)
    a('--nerf_length_max', type=float, default=25.5)
    a('--nerf_width_min', type=float, default=-4.5)
    a('--nerf_width_max', type=float, default=25.5)
    a('--nerf_height_min', type=float, default=-2.0)
    a('--nerf_height_max', type=float, default=0.5)
    # model (:64-78)
    a('--L_pos', type=int, default=10)
    a('--feature_size', type=int, default=256)
    a('--use_skip', default=True, action="store_true")
    a('--ckpt_path', type=str, default=None)
    a('--exp_name', type=str, default='nof_kitti/sequence00')
    a('--seed', type=int, default=42)
    a('--loss_type', type=str, default='smoothl1')
    # optimisation (:80-102)
    a('--batch_size', type=int, default=256)
    a('--batch_size_val', type=int, default=12)
    a('--optimizer', type=str, default='adam')
    a('--lr', type=float, default=5e-4)
    a('--momentum', type=float, default=0.9)
    a('--weight_decay', type=float, default=0)
    a('--chunk', type=int, default=32 * 1024)
    a('--num_epochs', type=int, default=16)
    a('--decay_step', nargs='+', type=int, default=[200])
    a('--decay_epochs', nargs='+', type=int, default=[2])
    a('--decay_gamma', type=float, default=0.1)
    # PC-NeRF losses and sampling (:104-130)
    a('--use_child_nerf_divide', type=int, default=0)
    a('--use_child_nerf_loss', type=int, default=0)
    a('--use_segmentated_sample', type=int, default=0)
    a('--segmentated_child_nerf_ratio', type=float, default=0.5)
    a('--lambda_loss', type=float, default=0.5)
    a('--lambda_loss_fine', type=float, default=0.5)
    a('--lambda_child_free_loss', type=float, default=0.5)
    a('--lambda_child_depth_loss', type=float, default=0.5)
    a('--N_samples', type=int, default=128)
    a('--N_importance', type=int, default=256)
    a('--perturb', type=float, default=1.0)
    a('--noise_std', type=float, default=0.0)
    a('--use_disp', default=False, action="store_true")
    # logging (:132-150)
    a('--visualize', type=int, default=1)
    a('--current_epoch', type=int, default=0)
    for k in ('', '_range', '_range_fine', '_child_free', '_child_free_fine', '_child_depth', '_child_depth_fine'):
        a(f'--saveploty_path{k}', type=str, default=None)
    a('--prefixes_to_ignore', nargs='+', type=str, default=['loss'])
    # this implementation only
    a('--device', type=str, default='cuda')
    a('--frame_sparsity', type=int, default=20, help="train-frame rule of ipb2dmapping.py:632-640 (percent)")
    a('--max_steps', type=int, default=0, help="stop after this many training steps (0: run every epoch)")
    a('--log_path', type=str, default=None, help="JSON-lines log of every step / validation")
    return p


def get_opts(argv=None):
    return build_parser().parse_args(argv)


def get_learning_rate(optimizer):
    for param_group in optimizer.param_groups:
        return param_group['lr']


def get_optimizer(hparams, parameters):
    """nof_utils.py:158-173: SGD(momentum) or Adam(eps 1e-8), both with weight decay."""
    if hparams.optimizer == 'sgd':
        return SGD(parameters, lr=hparams.lr, momentum=hparams.momentum, weight_decay=hparams.weight_decay)
    if hparams.optimizer == 'adam':
        return Adam(parameters, lr=hparams.lr, eps=1e-8, weight_decay=hparams.weight_decay)
    raise ValueError('optimizer not recognized!')


def decode_batch(batch):
    return batch['rays'], batch['ranges']


def decode_batch2(batch):
    return batch['rays']
