"""Compatibility import path (reference: atorch/atorch/common/)."""
