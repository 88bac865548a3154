"""``dgl.init`` (dataloader.py:215, 245)."""
from ..graph import zero_initializer  # noqa: F401
