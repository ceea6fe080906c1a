"""Compatibility import path (reference: atorch/atorch/modules/distributed_modules/)."""
