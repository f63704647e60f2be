"""ddp_practice_amd — MI355X-native single-node DDP + AMP training framework."""
__version__ = "0.1.0"
