from .loss import *  # noqa: F401,F403
from .loss import NOFMSELoss, NOFL1Loss, NOFSmoothL1Loss

nof_loss = {
    'mse': NOFMSELoss,
    'l1': NOFL1Loss,
    'smoothl1': NOFSmoothL1Loss,
}
