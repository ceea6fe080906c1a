"""ATorch capabilities re-designed for MI355X: auto_accelerate, parallel strategies,
fused-op modules, optimizers, data loaders, trainer, RL (reference: atorch/atorch)."""
