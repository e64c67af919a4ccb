"""Latency benchmark + report (reference: examples/inference/modules/benchmark.py:9-72; same report
schema: latency_ms_p50/p90/p95/p99/p100/avg and throughput = runs * max_length * batch / time).

GPU timing brackets each run with a device synchronisation so the host clock measures completed
work (the model calls already synchronise at the end of `generate`)."""

from __future__ import annotations

import time
from functools import partial

import numpy as np
import torch

BENCHMARK_REPORT_FILENAME = "benchmark_report.json"


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class LatencyCollector:
    def __init__(self):
        self.start = None
        self.latency_list = []

    def pre_hook(self, *args):
        _sync()
        self.start = time.perf_counter()

    def hook(self, *args):
        _sync()
        self.latency_list.append(time.perf_counter() - self.start)


class Benchmark:
    def __init__(self, benchmark_func, input_param, config, num_runs: int = 20, preprocess_func=None,
                 post_warmup_func=None):
        if isinstance(input_param, (tuple, list)):
            self.benchmark_func = partial(benchmark_func, *input_param)
        elif isinstance(input_param, dict):
            self.benchmark_func = partial(benchmark_func, **input_param)
        else:
            self.benchmark_func = partial(benchmark_func, input_param)
        self.config = config
        self.num_runs = num_runs
        self.preprocess_func = preprocess_func
        self.post_warmup_func = post_warmup_func
        self.latency_list = None

    def run(self):
        if self.preprocess_func:
            self.preprocess_func()
        self.benchmark_func()  # warm-up (graph capture, allocator pools)
        if self.post_warmup_func:
            self.post_warmup_func()
        lc = LatencyCollector()
        for _ in range(self.num_runs):
            if self.preprocess_func:
                self.preprocess_func()
            lc.pre_hook()
            self.benchmark_func()
            lc.hook()
        self.latency_list = lc.latency_list
        return self.latency_list


def generate_report(latency_list, config, max_length=None, batch_size=None):
    lat = np.array(latency_list)
    n = len(latency_list)
    max_length = max_length or config.generation_config["max_length"]
    batch_size = batch_size or config.max_batch_size
    return {
        "latency_ms_p50": float(np.percentile(lat, 50) * 1000),
        "latency_ms_p90": float(np.percentile(lat, 90) * 1000),
        "latency_ms_p95": float(np.percentile(lat, 95) * 1000),
        "latency_ms_p99": float(np.percentile(lat, 99) * 1000),
        "latency_ms_p100": float(np.percentile(lat, 100) * 1000),
        "latency_ms_avg": float(np.average(lat) * 1000),
        "throughput": float(n * max_length * batch_size / np.sum(lat)),
    }
