"""MNIST classifier forward + training step at batch 8192 (for rocprofv3 kernel stats)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from fet_ode_amd import mnist
from oracle import mnist_ref as M
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = mnist.KuramotoKANClassifier().to(dev)
x = M.mnist_x(8192, seed=3).to(dev)
y = (torch.arange(8192) % 10).to(dev)
with torch.no_grad():
    for _ in range(5):
        m(x)
for _ in range(3):
    m.zero_grad(set_to_none=True)
    torch.nn.functional.cross_entropy(m(x), y).backward()
torch.cuda.synchronize()
print("done")
