"""Compatibility module for ``from model.CANNet import CANNet`` (reference layout)."""
from can_distributed_pytorch_amd.models.cannet import CANNet, make_layers  # noqa: F401


if __name__ == "__main__":
    # model smoke test (reference model/CANNet.py:125-129): forward of ones(1,3,256,256), print the mean
    import torch
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    net = CANNet().to(dev)
    with torch.no_grad():
        out = net(torch.ones(1, 3, 256, 256, device=dev))
    print(tuple(out.shape), float(out.float().mean()))
