"""A TorchScript archive with the exported model's module tree (the
reference's export, M/model/deploy.py:77-121: ScriptableAdapter.model =
GeneralizedRCNN, Detectron2 parameter / buffer names, FastRCNNOutputLayers'
test thresholds as attributes), written with torch.jit.save for the import
tests."""
import torch


class Node(torch.nn.Module):
    def __init__(self):
        super().__init__()


class Adapter(torch.nn.Module):
    def __init__(self, sd, scalars):
        super().__init__()
        root = Node()
        self.add_module("model", root)
        for k, v in sd.items():
            parts = k.split(".")
            m = root
            for p in parts[:-1]:
                if p not in m._modules:
                    m.add_module(p, Node())
                m = m._modules[p]
            if k.endswith(("running_mean", "running_var")) or k.startswith("pixel"):
                m.register_buffer(parts[-1], v.clone())
            else:
                m.register_parameter(parts[-1], torch.nn.Parameter(v.clone(), requires_grad=False))
        for k, v in scalars.items():
            parts = k.split(".")
            m = root
            for p in parts[:-1]:
                m = m._modules[p]
            setattr(m, parts[-1], v)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x


def write_archive(path, sd, scalars):
    torch.jit.save(torch.jit.script(Adapter(sd, scalars)), str(path))
    return str(path)
