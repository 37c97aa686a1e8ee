"""MI355X-native drop-in for the reference's ``nof`` package (PC-NeRF render + loss hot path).

Put ``pc-nerf_amd/`` on ``sys.path`` (where the reference's repository root would be) and the reference drivers'
imports -- ``from nof.render import render_rays_train``, ``from nof.networks import NOF_coarse, Embedding``,
``from nof.criteria import nof_loss`` -- resolve here.  Compute runs in lib/libpcnerf_hip.so (gfx950).
"""
