from .models import NOF, Embedding, NOF_fine, NOF_coarse, NOF_plusfine  # noqa: F401
