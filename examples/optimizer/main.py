"""AGD / WSAM on an image classifier (reference: atorch/examples/optimizer/
main.py): a CIFAR-shaped ResNet trained with SGD, Adam(W), AGD or any of
them wrapped by Weighted SAM (closure-based two-pass step).

    python examples/optimizer/main.py --optimizer wsam --base_optimizer agd --lr 1e-3 --use-gpu
    python examples/optimizer/main.py --optimizer vanilla --base_optimizer agd --epochs 10

Data: 32x32x3 images of ``--classes`` random "prototype" patterns plus
noise (no download); the loss and accuracy must improve within an epoch.
"""

import argparse
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.utils.data import DataLoader, TensorDataset  # noqa: E402

from atorch.optimizers import AGD, WeightedSAM  # noqa: E402


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.short = nn.Sequential()
        if stride != 1 or cin != cout:
            self.short = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        return F.relu(self.b2(self.c2(y)) + self.short(x))


class ResNet(nn.Module):
    """CIFAR ResNet-(6n+2) (``--depth``)."""

    def __init__(self, depth=8, classes=10, width=16):
        super().__init__()
        n = (depth - 2) // 6
        self.stem = nn.Sequential(nn.Conv2d(3, width, 3, 1, 1, bias=False), nn.BatchNorm2d(width), nn.ReLU())
        layers, cin = [], width
        for i, w in enumerate((width, 2 * width, 4 * width)):
            for j in range(n):
                layers.append(BasicBlock(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        return self.fc(F.adaptive_avg_pool2d(self.layers(self.stem(x)), 1).flatten(1))


def synthetic_images(n, classes, seed=0):
    g = torch.Generator().manual_seed(seed)
    protos = torch.randn(classes, 3, 32, 32, generator=g)
    y = torch.randint(0, classes, (n,), generator=g)
    x = protos[y] + 1.5 * torch.randn(n, 3, 32, 32, generator=g)
    return TensorDataset(x, y)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--samples", type=int, default=2048)
    p.add_argument("--classes", type=int, default=10)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--weight-decay", type=float, default=5e-4)
    p.add_argument("--depth", type=int, default=8)
    p.add_argument("--optimizer", default="vanilla", choices=["vanilla", "wsam"])
    p.add_argument("--base_optimizer", default="sgd", choices=["sgd", "adam", "adamw", "agd"])
    p.add_argument("--eps", type=float, default=1e-8)
    p.add_argument("--adaptive", action="store_true")
    p.add_argument("--rho", type=float, default=0.05)
    p.add_argument("--gamma", type=float, default=0.5)
    p.add_argument("--mode", default="decouple", choices=["couple", "decouple"])
    p.add_argument("--use-gpu", action="store_true")
    p.add_argument("--seed", type=int, default=1)
    return p.parse_args(argv)


def build_optimizer(model, a):
    params = model.parameters()
    if a.base_optimizer == "sgd":
        base = torch.optim.SGD(params, lr=a.lr, momentum=0.9, weight_decay=a.weight_decay)
    elif a.base_optimizer == "adam":
        base = torch.optim.Adam(params, lr=a.lr, weight_decay=a.weight_decay)
    elif a.base_optimizer == "adamw":  # decoupled decay: rescale as the reference does
        base = torch.optim.AdamW(params, lr=a.lr, weight_decay=a.weight_decay / a.lr)
    else:
        base = AGD(params, lr=a.lr, delta=a.eps, weight_decay=a.weight_decay / a.lr)
    if a.optimizer == "vanilla":
        return base
    return WeightedSAM(model, base, rho=a.rho, gamma=a.gamma, adaptive=a.adaptive, decouple=a.mode == "decouple")


def main(argv=None):
    a = parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    torch.manual_seed(a.seed)
    dev = torch.device("cuda") if a.use_gpu and torch.cuda.is_available() else torch.device("cpu")
    model = ResNet(a.depth, a.classes).to(dev)
    opt = build_optimizer(model, a)
    loader = DataLoader(synthetic_images(a.samples, a.classes, a.seed), batch_size=a.batch_size, shuffle=True,
                        drop_last=True)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(getattr(opt, "base_optimizer", opt),
                                                       T_max=a.epochs * len(loader))
    crit = nn.CrossEntropyLoss()
    hist, step = [], 0
    for ep in range(a.epochs):
        t0, tot, correct, loss_sum = time.time(), 0, 0, 0.0
        for x, y in loader:
            x, y = x.to(dev), y.to(dev)
            if a.optimizer == "wsam":
                def closure():
                    loss = crit(model(x), y)
                    loss.backward()
                    return loss

                loss = opt.step(closure)
                out = None
            else:
                out = model(x)
                loss = crit(out, y)
                loss.backward()
                opt.step()
            opt.zero_grad()
            sched.step()
            loss_sum += float(loss) * y.numel()
            tot += y.numel()
            if out is not None:
                correct += int((out.argmax(1) == y).sum())
            hist.append(float(loss))
            step += 1
            if a.max_steps and step >= a.max_steps:
                break
        logging.info(f"epoch {ep}: loss {loss_sum / tot:.4f}"
                     + (f" acc {correct / tot:.3f}" if a.optimizer != "wsam" else "")
                     + f" ({time.time() - t0:.1f}s, {a.optimizer}/{a.base_optimizer})")
    print(f"first_loss={hist[0]:.4f} last_loss={sum(hist[-5:]) / len(hist[-5:]):.4f}", flush=True)
    return hist


if __name__ == "__main__":
    main()
