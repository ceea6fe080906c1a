"""Compatibility import path (reference: atorch/atorch/auto/opt_lib/)."""
