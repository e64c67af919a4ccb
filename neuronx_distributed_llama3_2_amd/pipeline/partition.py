"""Partition a traced model into pipeline stages
(reference: src/neuronx_distributed/pipeline/partition.py:18-303).

Cuts are placed before chosen transformer-layer calls; every graph node is assigned to the stage
of the last cut preceding it, and `torch.fx.passes.split_module` builds one sub-GraphModule per
stage.  `analyze_pipeline_module` reads the wiring graph to find, for every stage, which model
inputs it reads, which values it receives from earlier stages (including values that have to be
passed THROUGH intermediate stages because only neighbours exchange data), and what it sends on.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Set

import torch
import torch.fx as fx
from torch.fx.passes.split_module import split_module


def create_partitions(num_stages: int, num_layers: int) -> List[int]:
    """Indices of the layers that START stages 1..n-1; layers spread evenly, remainder to later stages."""
    base, rem = divmod(num_layers, num_stages)
    sizes = [base + (1 if s >= num_stages - rem else 0) for s in range(num_stages)]
    starts, acc = [], 0
    for s in sizes[:-1]:
        acc += s
        starts.append(acc)
    return starts


def stage_to_pipeline_parallel_rank(stage: int, pipeline_parallel_size: int) -> int:
    return stage % pipeline_parallel_size


def partition_traced_model(gm: fx.GraphModule, cut_layer_names: Sequence[str]) -> fx.GraphModule:
    """Split `gm` before each call_module node whose target is in `cut_layer_names`."""
    cuts = set(cut_layer_names)
    stage_of: Dict[fx.Node, int] = {}
    cur = 0
    for node in gm.graph.nodes:
        if node.op == "call_module" and node.target in cuts:
            cur += 1
        stage_of[node] = cur
    missing = cuts - {n.target for n in gm.graph.nodes if n.op == "call_module"}
    if missing:
        raise ValueError(f"pipeline cut points not found in the traced graph: {sorted(missing)}")

    def cb(node):
        return stage_of[node]

    return split_module(gm, gm, cb, keep_original_order=True)


@dataclass
class PipelineIO:
    stage: int
    model_inputs: List[str] = field(default_factory=list)   # placeholders read from the batch
    inputs: List[str] = field(default_factory=list)         # ordered argument names of the stage submodule
    recv: List[str] = field(default_factory=list)           # values received from the previous stage
    send: List[str] = field(default_factory=list)           # values sent to the next stage
    outputs: List[str] = field(default_factory=list)        # values this stage's submodule produces
    is_last: bool = False


def analyze_pipeline_module(split_gm: fx.GraphModule, num_stages: int) -> List[PipelineIO]:
    """Stage IO from the wiring graph of a split GraphModule."""
    g = split_gm.graph
    placeholders = [n.name for n in g.nodes if n.op == "placeholder"]
    produced_by: Dict[str, int] = {}
    ios = [PipelineIO(s) for s in range(num_stages)]
    stage_nodes: Dict[int, fx.Node] = {}
    getitem_src: Dict[str, str] = {}
    for n in g.nodes:
        if n.op == "call_module" and n.target.startswith("submod_"):
            s = int(n.target.split("_")[1])
            stage_nodes[s] = n
    # every value node in the wiring graph: placeholder, submod call, getitem of a submod call
    for n in g.nodes:
        if n.op == "call_module" and n.target.startswith("submod_"):
            s = int(n.target.split("_")[1])
            produced_by[n.name] = s
        elif n.op == "call_function" and n.target.__name__ == "getitem" and n.args[0].name in produced_by:
            produced_by[n.name] = produced_by[n.args[0].name]
            getitem_src[n.name] = n.args[0].name
    consumers: Dict[str, Set[int]] = {}
    for s, node in stage_nodes.items():
        args = []
        for a in node.args:
            assert isinstance(a, fx.Node), "stage submodule arguments must be graph values"
            args.append(a.name)
            if a.name in placeholders:
                ios[s].model_inputs.append(a.name)
            consumers.setdefault(a.name, set()).add(s)
        ios[s].inputs = args
    out_node = [n for n in g.nodes if n.op == "output"][0]
    final_values = [a.name for a in _flatten_nodes(out_node.args)]
    last = num_stages - 1
    for v in final_values:
        consumers.setdefault(v, set()).add(last + 1)  # the model output is consumed "after" the last stage
    for v, cons in consumers.items():
        if v not in produced_by:
            continue
        src = produced_by[v]
        dst = max(cons)
        if dst == last + 1:
            dst = last
        for s in range(src, dst):
            if v not in ios[s].send:
                ios[s].send.append(v)
            if v not in ios[s + 1].recv:
                ios[s + 1].recv.append(v)
    for s, node in stage_nodes.items():
        ios[s].outputs = [n for n, p in produced_by.items() if p == s]
    ios[last].is_last = True
    return ios


def _flatten_nodes(arg) -> List[fx.Node]:
    out: List[fx.Node] = []

    def visit(a):
        if isinstance(a, fx.Node):
            out.append(a)
        elif isinstance(a, (list, tuple)):
            for x in a:
                visit(x)
        elif isinstance(a, dict):
            for x in a.values():
                visit(x)

    visit(arg)
    return out


def analyze_shared_weights_across_stages(split_gm: fx.GraphModule, num_stages: int) -> List[List[tuple]]:
    """Parameters (by identity) used by more than one stage: [[(stage, qualified name), ...], ...]."""
    owners: Dict[int, List[tuple]] = {}
    for s in range(num_stages):
        sub = getattr(split_gm, f"submod_{s}", None)
        if sub is None:
            continue
        for name, p in sub.named_parameters(remove_duplicate=False):
            owners.setdefault(id(p), []).append((s, name))
    return [v for v in owners.values() if len({s for s, _ in v}) > 1]
