"""Inference runner: trace (compile) -> load -> generate / check accuracy / benchmark
(reference: examples/inference/runner.py:46-655 `InferenceRunner`, llama3/llama3_runner.py).

    r = InferenceRunner(model_path=hf_dir, tokenizer_path=hf_dir)
    r.trace(traced_path, tp_degree=1, batch_size=1, max_prompt_length=128, sequence_length=256)
    model = r.load_neuron_model(traced_path)
    outs = r.generate_on_neuron(["Hello"], model, max_length=64)
    r.check_accuracy(model, prompts=[...])             # greedy tokens == HF transformers (CPU fp32)
    r.benchmark_sampling(model)                        # benchmark_report.json

Prompts may be strings (needs a local tokenizer: there is no network) or token-id lists.
Everything runs one process per GPU; with tp_degree > 1 launch under torchrun (SPMD).
"""

from __future__ import annotations

import json
import os
from contextlib import contextmanager
from typing import Dict, List, Optional, Sequence, Union

import torch

from .benchmark import BENCHMARK_REPORT_FILENAME, Benchmark, LatencyCollector, generate_report
from .config import InferenceConfig, model_config_from_dir
from .generation import LlamaForCausalLMInference

Prompt = Union[str, Sequence[int]]


class InferenceRunner:
    app_cls = LlamaForCausalLMInference   # the inference application this runner drives

    def __init__(self, model_path: Optional[str] = None, tokenizer_path: Optional[str] = None,
                 generation_config: Optional[dict] = None):
        self.model_path = model_path
        self.tokenizer_path = tokenizer_path
        self.generation_config = dict(generation_config or {})
        self._profile = False
        self.config: Optional[InferenceConfig] = None

    # ------------------------------------------------------------------ construction
    def get_config_for_nxd(self, batch_size: int, tp_degree: int, max_prompt_length: int, sequence_length: int,
                           enable_bucketing: bool = False, **kwargs) -> InferenceConfig:
        return InferenceConfig(tp_degree=tp_degree, batch_size=batch_size, seq_len=sequence_length,
                               max_context_length=max_prompt_length, enable_bucketing=enable_bucketing, **kwargs)

    def load_hf_model(self):
        from transformers import LlamaForCausalLM

        return LlamaForCausalLM.from_pretrained(self.model_path, torch_dtype=torch.float32).eval()

    def load_tokenizer(self, padding_side: Optional[str] = None):
        if not self.tokenizer_path or not any(
                os.path.exists(os.path.join(self.tokenizer_path, f))
                for f in ("tokenizer.json", "tokenizer.model", "tokenizer_config.json")):
            return None
        from transformers import AutoTokenizer

        try:
            tok = AutoTokenizer.from_pretrained(self.tokenizer_path, local_files_only=True)
        except Exception:   # no usable tokenizer files: token-id prompts only
            return None
        tok.padding_side = padding_side or "right"
        if tok.pad_token is None:
            tok.pad_token = tok.eos_token
        return tok

    def load_neuron_model_on_cpu(self, max_prompt_length: int, sequence_length: int, batch_size: int, **kwargs):
        cfg = self.get_config_for_nxd(batch_size, 1, max_prompt_length, sequence_length, **kwargs)
        cfg.use_hip_graphs = False
        m = self.app_cls.from_pretrained(self.model_path, cfg, dtype=torch.float32)
        return m

    def trace(self, traced_model_path: str, tp_degree: int = 1, batch_size: int = 1, max_prompt_length: int = 128,
              sequence_length: int = 256, enable_bucketing: bool = False, **kwargs) -> None:
        """Shard the HF weights for every rank and write them + the configs (the reference's
        trace/compile step; kernels are prebuilt, graphs are captured at load)."""
        self.config = self.get_config_for_nxd(batch_size, tp_degree, max_prompt_length, sequence_length,
                                              enable_bucketing, **kwargs)
        m = self.app_cls.from_pretrained(self.model_path, self.config)
        m.compile(traced_model_path)
        if self.tokenizer_path and os.path.isdir(self.tokenizer_path):
            tok = self.load_tokenizer()
            if tok is not None and (not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0):
                tok.save_pretrained(traced_model_path)

    def load_neuron_model(self, traced_model_path: str):
        """In-process model; a traced model with tp_degree > 1 loaded without torch.distributed
        (plain `python`, no launcher) is served by resident per-GPU workers instead
        (inference/spmd_server.py: one controller, ids in / ids out)."""
        import torch.distributed as dist

        cfg = InferenceConfig.from_pretrained(traced_model_path)
        if int(cfg.tp_degree) > 1 and not dist.is_initialized():
            from .spmd_server import SpmdGenerationServer

            app = "llama" if self.app_cls is LlamaForCausalLMInference else self.app_cls.__name__
            m = SpmdGenerationServer.from_compiled(traced_model_path, int(cfg.tp_degree), app=app)
            self.config = m.config
            return m
        m = self.app_cls.load(traced_model_path)
        self.config = m.config
        return m

    # ------------------------------------------------------------------ generation
    def _encode(self, prompts: Sequence[Prompt], tokenizer=None):
        if prompts and isinstance(prompts[0], str):
            tokenizer = tokenizer or self.load_tokenizer()
            assert tokenizer is not None, "string prompts need a local tokenizer (tokenizer_path)"
            enc = tokenizer(list(prompts), return_tensors="pt", padding=True)
            return enc["input_ids"], enc["attention_mask"]
        L = max(len(p) for p in prompts)
        ids = torch.zeros((len(prompts), L), dtype=torch.long)
        mask = torch.zeros_like(ids)
        for i, p in enumerate(prompts):
            ids[i, :len(p)] = torch.as_tensor(list(p))
            mask[i, :len(p)] = 1
        return ids, mask

    def generate_on_neuron(self, prompts: Sequence[Prompt], model: LlamaForCausalLMInference, draft_model=None,
                           max_length: Optional[int] = None, **kwargs) -> torch.Tensor:
        ids, mask = self._encode(prompts)
        gen = dict(self.generation_config)
        gen.update(kwargs)
        max_new = (max_length or model.config.max_length) - ids.shape[1]
        with self._maybe_profile():
            return model.generate(ids, mask, max_new_tokens=max_new, assistant_model=draft_model, **gen).cpu()

    def generate_on_cpu(self, prompts: Sequence[Prompt], batch_size: int, max_prompt_length: int, sequence_length: int,
                        **kwargs) -> torch.Tensor:
        m = self.load_neuron_model_on_cpu(max_prompt_length, sequence_length, batch_size)
        return self.generate_on_neuron(prompts, m, max_length=sequence_length, **kwargs)

    def generate_with_hf(self, prompts: Sequence[Prompt], max_length: int, **kwargs) -> torch.Tensor:
        ids, mask = self._encode(prompts)
        hf = self.load_hf_model()
        out = []
        with torch.no_grad():   # greedy, one sequence at a time (right padding is not HF-generate friendly)
            for i in range(ids.shape[0]):
                n = int(mask[i].sum())
                o = hf.generate(ids[i:i + 1, :n], attention_mask=mask[i:i + 1, :n], max_length=max_length,
                                do_sample=False, pad_token_id=hf.config.eos_token_id or 0, **kwargs)
                out.append(o[0])
        return out

    def check_accuracy(self, model: LlamaForCausalLMInference, prompts: Sequence[Prompt],
                       max_length: Optional[int] = None, num_tokens_to_check: Optional[int] = None) -> bool:
        """Greedy tokens of `model` == HF transformers (CPU fp32) on the same prompts."""
        max_length = max_length or model.config.max_length
        ref = self.generate_with_hf(prompts, max_length)
        ids, mask = self._encode(prompts)
        got = model.generate(ids, mask, max_new_tokens=max_length - ids.shape[1], eos_token_id=None).cpu()
        ok = True
        for i, r in enumerate(ref):
            n = int(mask[i].sum())
            new_ref = r[n:]
            new_got = got[i, ids.shape[1]:ids.shape[1] + len(new_ref)]
            k = num_tokens_to_check or len(new_ref)
            if not torch.equal(new_ref[:k], new_got[:k]):
                ok = False
        return ok

    def check_accuracy_logits(self, model: LlamaForCausalLMInference, prompts: Sequence[Prompt],
                              rtol: float = 3e-2) -> float:
        """Max relative difference of the prefill logits against HF transformers."""
        ids, mask = self._encode(prompts)
        hf = self.load_hf_model()
        with torch.no_grad():
            ref = hf(input_ids=ids, attention_mask=mask).logits
        lengths = mask.sum(1)
        ref_last = ref[torch.arange(ids.shape[0]), lengths - 1]
        got = model._context_encode(ids, mask).cpu().float()
        err = float((got - ref_last).abs().max() / ref_last.abs().max())
        return err

    # ------------------------------------------------------------------ benchmarking / profiling
    def benchmark_sampling(self, model: LlamaForCausalLMInference, draft_model=None, num_runs: int = 20,
                           prompt_len: Optional[int] = None, report_path: Optional[str] = None) -> Dict[str, dict]:
        cfg = model.config
        B = cfg.max_batch_size
        T = prompt_len or cfg.max_context_length
        g = torch.Generator().manual_seed(0)
        ids = torch.randint(3, model.model_config.vocab_size, (B, T), generator=g)
        max_new = cfg.max_length - T

        def e2e():
            model.generate(ids, max_new_tokens=max_new, eos_token_id=None, assistant_model=draft_model)

        bench = Benchmark(e2e, (), cfg, num_runs=num_runs)
        lat = bench.run()
        report = {"e2e_model": generate_report(lat, cfg, max_length=cfg.max_length, batch_size=B)}
        # sub-model latencies through the context-encoding / token-generation wrappers
        ce = LatencyCollector()
        model.context_encoding_model.register_forward_pre_hook(ce.pre_hook)
        model.context_encoding_model.register_forward_hook(ce.hook)
        for _ in range(max(3, num_runs // 4)):
            model.context_encoding_model(ids)
        report["context_encoding_model"] = generate_report(ce.latency_list, cfg, max_length=T, batch_size=B)
        path = report_path or BENCHMARK_REPORT_FILENAME
        with open(path, "w") as f:
            json.dump(report, f, indent=2)
        return report

    def enable_torch_profile(self):
        self._profile = True

    def is_torch_profile_enabled(self) -> bool:
        return self._profile

    @contextmanager
    def torch_profile(self, chrome_trace_path: str = "torch-trace.json", **profile_kwargs):
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
        with profile(activities=acts, **profile_kwargs) as p:
            yield p
        p.export_chrome_trace(chrome_trace_path)

    @contextmanager
    def _maybe_profile(self):
        if self._profile:
            with self.torch_profile():
                yield
        else:
            yield


class LlamaRunner(InferenceRunner):
    """Llama-3 / 3.1 / 3.2 runner (reference: examples/inference/llama3/llama3_runner.py)."""

    def get_padding_side(self):
        return "right"
