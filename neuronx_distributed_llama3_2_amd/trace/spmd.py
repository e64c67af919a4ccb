"""SPMD inference runtime pieces: per-bucket hipGraph runners, the shape router, state
initialisation (reference: src/neuronx_distributed/trace/spmd.py:9-187 — SPMDBucketModel,
StateInitializer, NxDModel, NxDModelExecutor on top of torch_neuronx SPMDModel / NEFFs).

MI355X design: "compiling" a bucket = capturing the module's forward for that input shape into a
hipGraph (kernels are prebuilt HIP; the graph removes per-kernel launch cost and host work).
Inputs are copied into the graph's static input buffers, the graph replays, outputs are returned
as copies.  State tensors (e.g. KV caches) are ordinary module buffers updated in place, which is
the reference's input/output aliasing without any alias bookkeeping.  One process per GPU: every
rank holds its own NxDModel over its weight shard (SPMD); trace/runtime.py adds a single-
controller front end that drives one worker process per GPU.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import torch
from ..utils.graph_capture import graph_capture


def _shape_key(inputs: Sequence[torch.Tensor]) -> str:
    return str([tuple(t.shape) for t in inputs])


class GraphRunner:
    """One captured bucket: static inputs, graph, static outputs."""

    def __init__(self, fn: Callable, example_inputs: Sequence[torch.Tensor], use_graph: bool = True, warmup: int = 2):
        self.fn = fn
        self.static_in = [t.clone() for t in example_inputs]
        dev = self.static_in[0].device if self.static_in else torch.device("cpu")
        self.graph = None
        self.static_out = None
        if use_graph and dev.type == "cuda":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(warmup):     # allocator pools, GEMM tuning, lazy kernel loads
                    fn(*self.static_in)
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with graph_capture(self.graph):
                self.static_out = fn(*self.static_in)

    def __call__(self, *inputs: torch.Tensor):
        if self.graph is None:
            return self.fn(*inputs)
        for dst, src in zip(self.static_in, inputs):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        out = self.static_out
        if isinstance(out, torch.Tensor):
            return out.clone()
        return type(out)(o.clone() if isinstance(o, torch.Tensor) else o for o in out)


class SPMDBucketModel(torch.nn.Module):
    """All buckets (input shapes) of ONE model key on this rank."""

    def __init__(self, module: torch.nn.Module, example_inputs: List[Sequence[torch.Tensor]], use_graph: bool = True,
                 forward_fn: Optional[Callable] = None):
        super().__init__()
        self.module = module
        self.example_inputs = list(example_inputs)
        self.use_graph = use_graph
        self.forward_fn = forward_fn or module
        self.runners: Dict[str, GraphRunner] = {}

    def build(self) -> None:
        for ex in self.example_inputs:
            self.runners[_shape_key(ex)] = GraphRunner(self.forward_fn, ex, self.use_graph)

    def shape_keys(self) -> List[str]:
        return [_shape_key(ex) for ex in self.example_inputs]

    def forward(self, *inputs: torch.Tensor):
        r = self.runners.get(_shape_key(inputs))
        if r is None:
            raise KeyError(f"no bucket traced for input shapes {_shape_key(inputs)}; "
                           f"have {list(self.runners)}")
        return r(*inputs)


SPMDBucketModelScript = SPMDBucketModel   # reference name of the scripted wrapper


class StateInitializer(torch.nn.Module):
    """Creates the (zeroed) state tensors of a model, e.g. KV caches, from shapes / dtypes."""

    def __init__(self, shapes: Dict[str, Sequence[int]], dtypes: Dict[str, torch.dtype], tp_degree: int = 1,
                 device=None):
        super().__init__()
        self.shapes, self.dtypes, self.tp_degree = dict(shapes), dict(dtypes), tp_degree
        self.device = device

    def forward(self) -> Dict[str, torch.Tensor]:
        dev = self.device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu")
        return {k: torch.zeros(tuple(s), dtype=self.dtypes[k], device=dev) for k, s in self.shapes.items()}


class NxDModel(torch.nn.Module):
    """Several bucketed models (e.g. context encoding + token generation) that share weights;
    `forward(inputs)` routes on the input shapes (or a user router) to the traced bucket."""

    def __init__(self, models: Dict[str, SPMDBucketModel], tp_degree: int = 1, router: Optional[Callable] = None,
                 state_initializer: Optional[StateInitializer] = None):
        super().__init__()
        self.models = torch.nn.ModuleDict(models)
        self.tp_degree = tp_degree
        self.user_router = router
        self.state_initializer = state_initializer
        self.state: Dict[str, torch.Tensor] = {}
        self.input_shape_map: Dict[str, str] = {}
        for key, m in models.items():
            for sk in m.shape_keys():
                self.input_shape_map.setdefault(sk, key)

    def _modules_unique(self) -> List[torch.nn.Module]:
        seen, out = set(), []
        for m in self.models.values():
            if id(m.module) not in seen:
                seen.add(id(m.module))
                out.append(m.module)
        return out

    def initialize(self, checkpoint: Dict[str, torch.Tensor], strict: bool = False) -> None:
        """Load THIS rank's weight shard into every (shared) module, create states, then capture."""
        for mod in self._modules_unique():
            dev = next((p.device for p in mod.parameters()), None)
            if dev is not None and dev.type == "meta":
                mod.to_empty(device=torch.device("cuda", torch.cuda.current_device())
                             if torch.cuda.is_available() else torch.device("cpu"))
            mod.load_state_dict(checkpoint, strict=strict)
        self.initialize_with_saved_weights()

    def initialize_with_saved_weights(self) -> None:
        if self.state_initializer is not None:
            self.state = self.state_initializer()
        for m in self.models.values():
            m.build()

    def router(self, inputs: Sequence[torch.Tensor]) -> str:
        if self.user_router is not None:
            return self.user_router(inputs)
        key = self.input_shape_map.get(_shape_key(inputs))
        if key is None:
            raise KeyError(f"no traced model accepts input shapes {_shape_key(inputs)}")
        return key

    def forward(self, inputs: List[torch.Tensor]):
        return self.models[self.router(inputs)](*inputs)


class NxDModelExecutor(torch.nn.Module):
    """`model(*inputs)` front end over NxDModel (reference spmd.py:177-187)."""

    def __init__(self, nxd_model):
        super().__init__()
        self.nxd_model = nxd_model

    def forward(self, *inputs):
        return self.nxd_model(list(inputs))
