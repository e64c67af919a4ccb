"""Example scripts run end-to-end on CPU (gloo): Llama TP+ZeRO-1 pre-training with checkpoint /
resume and the metrics file (reference examples E1)."""

import json
import os
import sys

import torch

from dist_utils import run_distributed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _w_pretrain(rank, world, out_dir, cfg_path, steps_this_run, data):
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "llama"))
    import tp_zero1_llama_hf_pretrain as ex

    argv = ["--model_path", cfg_path, "--tensor_parallel_size", "2", "--seq_len", "32", "--batch_size", "2",
            "--grad_accum_usteps", "2", "--max_steps", "4", "--steps_this_run", str(steps_this_run), "--use_zero_1",
            "--sequence_parallel_enabled", "--checkpoint_dir", os.path.join(out_dir, "ckpt"), "--checkpoint_freq",
            "2", "--output_dir", out_dir, "--lr", "1e-3", "--warmup_steps", "1"]
    if data:
        argv += ["--data_dir", data]
    loss = ex.main(argv)
    if rank == 0:
        torch.save(float(loss), os.path.join(out_dir, f"loss_{steps_this_run}.pt"))


def test_llama_pretrain_example_tp2_zero1_resume(tmp_path):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import llama_config
    from neuronx_distributed_llama3_2_amd.utils.data_loader import write_token_file

    cfg = llama_config("tiny", num_hidden_layers=2, hidden_size=64, intermediate_size=128, vocab_size=256,
                       num_attention_heads=4, num_key_value_heads=2)
    cfg_path = str(tmp_path / "config.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg.to_dict(), f)
    data = str(tmp_path / "tokens.bin")
    g = torch.Generator().manual_seed(0)
    write_token_file(data, [torch.randint(0, 256, (20000,), generator=g).numpy()])
    # world 4 = TP2 x DP2; 2 steps, checkpoint, then resume for the remaining 2
    run_distributed(_w_pretrain, 4, str(tmp_path), cfg_path, 2, data)
    assert os.path.isdir(tmp_path / "ckpt" / "step_2")
    run_distributed(_w_pretrain, 4, str(tmp_path), cfg_path, 2, data)
    assert os.path.isdir(tmp_path / "ckpt" / "step_4")
    m = json.load(open(tmp_path / "results.json"))
    names = {x["MetricName"] for x in m["results"]["metrics"]}
    assert "Average throughput" in names and m["results"]["parameters"]["tensor_parallel_size"] == 2
    assert torch.isfinite(torch.tensor(torch.load(tmp_path / "loss_2.pt")))


def test_inference_runner_cli_trace_generate_check(tmp_path):
    """examples/inference/llama3_2_runner.py on CPU: trace (shard + configs) -> load -> greedy
    generation == HF transformers (check_accuracy) -> benchmark report."""
    import importlib.util

    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=200, max_position_embeddings=128, tie_word_embeddings=True,
                      eos_token_id=2, bos_token_id=1, rope_theta=500000.0)
    torch.manual_seed(0)
    hf_dir = str(tmp_path / "hf")
    LlamaForCausalLM(cfg).save_pretrained(hf_dir)
    spec = importlib.util.spec_from_file_location("runner_cli", os.path.join(ROOT, "examples", "inference",
                                                                           "llama3_2_runner.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    traced = str(tmp_path / "traced")
    base = ["--model_path", hf_dir, "--traced_path", traced, "--max_prompt_length", "16", "--sequence_length", "40"]
    cli.main(["trace"] + base)
    assert os.path.exists(os.path.join(traced, "tp0_sharded_checkpoint.safetensors"))
    out = cli.main(["generate"] + base + ["--prompt_ids", "5,6,7,8"])
    assert out.shape == (1, 40)
    assert cli.main(["check_accuracy"] + base + ["--prompt_ids", "5,6,7,8,9,10"]) is True
    rep = cli.main(["benchmark"] + base + ["--num_runs", "2"])
    assert "e2e_model" in rep and rep["e2e_model"]["latency_ms_p50"] > 0


def test_moe_and_quantized_inference_clis(tmp_path):
    """examples/inference/run_dbrx.py and run_llama_quantized.py: trace an HF directory, reload,
    generate (reference examples E10/E11: run_dbrx.py, run_llama_quantized.py)."""
    sys.path.insert(0, os.path.join(ROOT, "examples", "inference"))
    import run_dbrx  # noqa: F401  (module import = the CLI wiring is valid)
    import run_llama_quantized
    from llama3_2_runner import main as runner_main
    from transformers import DbrxConfig, DbrxForCausalLM, LlamaConfig, LlamaForCausalLM

    from neuronx_distributed_llama3_2_amd.inference.moe import DbrxRunner

    torch.manual_seed(0)
    dbrx = DbrxForCausalLM(DbrxConfig(d_model=64, n_heads=4, n_layers=1, max_seq_len=128, vocab_size=128,
                                      attn_config=dict(kv_n_heads=2, clip_qkv=8.0, rope_theta=10000.0),
                                      ffn_config=dict(ffn_hidden_size=64, moe_num_experts=4, moe_top_k=2)))
    src = str(tmp_path / "dbrx")
    dbrx.save_pretrained(src)
    traced = str(tmp_path / "dbrx_traced")
    runner_main(["trace", "--model_path", src, "--traced_path", traced, "--max_prompt_length", "16",
                 "--sequence_length", "24"], runner_cls=DbrxRunner)
    out = runner_main(["generate", "--traced_path", traced, "--prompt_ids", "3,4,5"], runner_cls=DbrxRunner)
    assert out.shape == (1, 24)
    llama = LlamaForCausalLM(LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                                         num_attention_heads=4, num_key_value_heads=2, vocab_size=128,
                                         max_position_embeddings=128))
    lsrc = str(tmp_path / "llama")
    llama.save_pretrained(lsrc)
    q = run_llama_quantized.main(["--model_path", lsrc, "--traced_path", str(tmp_path / "q"), "--max_prompt_length",
                                  "16", "--sequence_length", "24", "--prompt_ids", "7,8,9"])
    assert q.shape == (1, 24)


def test_infill_transform_and_codegen_data_script(tmp_path):
    """CodeGen2.5 causal-infilling rewrite (reference: codegen25/get_dataset_infill.py): every
    masked span reappears after the separator, in order, terminated by <eom>; blocks keep their size."""
    import numpy as np

    from neuronx_distributed_llama3_2_amd.utils.training_utils import format_to_infill, infill_token_blocks

    MASKS, EOM, SEP = [1001, 1002, 1003], 1010, [1020, 1021]
    toks = list(range(40))
    out = format_to_infill(toks, 2, MASKS, EOM, SEP, np.random.default_rng(0))
    s = out.index(SEP[0])
    prefix, suffix = out[:s], out[s + 2:]
    assert prefix.count(MASKS[0]) == 1 and prefix.count(MASKS[1]) == 1
    spans = []
    for m in MASKS[:2]:
        i = suffix.index(m)
        j = suffix.index(EOM, i)
        spans.append(suffix[i + 1:j])
    # prefix with each hole filled by its span restores the original sequence
    rebuilt = []
    for t in prefix:
        rebuilt += spans[MASKS.index(t)] if t in MASKS else [t]
    assert rebuilt == toks
    assert format_to_infill(toks[:3], 3, MASKS, EOM, SEP, np.random.default_rng(0)) is None
    blocks = infill_token_blocks([list(range(64)) for _ in range(10)], 64, MASKS, EOM, SEP, seed=1)
    assert all(len(b) == 64 for b in blocks) and any(SEP[0] in b for b in blocks)
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "codegen25"))
    import get_dataset_infill

    from neuronx_distributed_llama3_2_amd.utils.data_loader import write_token_file

    src = str(tmp_path / "toks.bin")
    write_token_file(src, [np.arange(32 * 8) % 500])
    res = get_dataset_infill.main(["--input", src, "--output", str(tmp_path / "inf.bin"), "--block_size", "32",
                                   "--mask_ids", "1001,1002", "--eom_id", "1010", "--sep_ids", "1020,1021"])
    assert len(res) == 8 and np.fromfile(str(tmp_path / "inf.bin"), dtype=np.uint32).size == 256


def _w_family(rank, world, out_dir, family, extra):
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "llama"))
    import tp_zero1_llama_hf_pretrain as ex

    argv = ["--model_family", family, "--model_path", "tiny", "--tensor_parallel_size", "2", "--seq_len", "32",
            "--batch_size", "1", "--max_steps", "3", "--use_zero_1", "--sequence_parallel_enabled", "--output_dir",
            out_dir, "--lr", "1e-3", "--warmup_steps", "1"] + extra
    loss = ex.main(argv)
    if rank == 0:
        torch.save(float(loss), os.path.join(out_dir, f"{family}.pt"))


def test_pretrain_example_mixtral_and_neox_families(tmp_path):
    """The pre-training example drives the other model families (reference examples E4 Mixtral,
    E5 GPT-NeoX) with TP=2 + SP + ZeRO-1 on gloo."""
    for fam, extra in (("mixtral", []), ("gpt_neox", [])):
        run_distributed(_w_family, 2, str(tmp_path), fam, extra)
        loss = torch.load(str(tmp_path / f"{fam}.pt"))
        assert loss == loss and loss < 20.0


def _w_pp_pretrain(rank, world, out_dir, cfg_path, steps_this_run):
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "llama"))
    import tp_pp_llama_hf_pretrain as ex

    argv = ["--model_path", cfg_path, "--tensor_parallel_size", "2", "--pipeline_parallel_size", "2",
            "--num_microbatches", "2", "--train_batch_size", "4", "--seq_len", "32", "--max_steps", "4",
            "--steps_this_run", str(steps_this_run), "--use_zero_1", "--sequence_parallel_enabled",
            "--checkpoint_dir", os.path.join(out_dir, "ckpt"), "--checkpoint_freq", "2", "--output_dir", out_dir,
            "--lr", "1e-3", "--warmup_steps", "1", "--watchdog_timeout", "600"]
    loss = ex.main(argv)
    if rank == 0:
        torch.save(float(loss), os.path.join(out_dir, f"pp_loss_{steps_this_run}.pt"))


def test_llama_tp_pp_example_resume(tmp_path):
    """examples/training/llama/tp_pp_llama_hf_pretrain.py (reference E2): TP2 x PP2 1F1B with ZeRO-1
    and SP on 4 gloo ranks, checkpoint at step 2, resume to step 4."""
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import llama_config

    cfg = llama_config("tiny", num_hidden_layers=4, hidden_size=64, intermediate_size=128, vocab_size=256,
                       num_attention_heads=4, num_key_value_heads=2)
    cfg_path = str(tmp_path / "config.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg.to_dict(), f)
    run_distributed(_w_pp_pretrain, 4, str(tmp_path), cfg_path, 2)
    assert os.path.exists(tmp_path / "ckpt" / "step_2" / "done")
    run_distributed(_w_pp_pretrain, 4, str(tmp_path), cfg_path, 2)
    assert os.path.exists(tmp_path / "ckpt" / "step_4" / "done")
    assert torch.isfinite(torch.tensor(torch.load(tmp_path / "pp_loss_2.pt")))
    m = json.load(open(tmp_path / "results.json"))
    assert m["results"]["parameters"]["pipeline_parallel_size"] == 2


def _w_bert(rank, world, out_dir):
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "bert"))
    import tp_dp_bert_hf_pretrain as ex

    loss = ex.main(["--model", "tiny", "--tensor_parallel_size", "2", "--batch_size", "4", "--seq_len", "32",
                    "--max_steps", "6", "--warmup_steps", "1", "--lr", "2e-3", "--output_dir", out_dir,
                    "--grad_accum_usteps", "2"])
    if rank == 0:
        torch.save(float(loss), os.path.join(out_dir, "bert_loss.pt"))


def test_bert_tp_dp_example(tmp_path):
    """examples/training/bert/tp_dp_bert_hf_pretrain.py (reference E6): TP2 x DP2 MLM+NSP."""
    run_distributed(_w_bert, 4, str(tmp_path))
    assert torch.isfinite(torch.tensor(torch.load(tmp_path / "bert_loss.pt")))
    m = json.load(open(tmp_path / "results.json"))
    assert {x["MetricName"] for x in m["results"]["metrics"]} >= {"Final loss", "Average throughput"}


def _w_finetune(rank, world, hf_dir, data, out_dir, tp):
    sys.path.insert(0, os.path.join(ROOT, "examples", "training", "llama"))
    import tp_llama_hf_finetune as ex

    before, after = ex.main(["--hf_model_dir", hf_dir, "--data_file", data, "--output_dir", out_dir,
                             "--tensor_parallel_size", str(tp), "--seq_len", "64", "--max_steps", "40",
                             "--lr", "1e-2", "--warmup_steps", "2", "--test_size", "4", "--use_zero_1",
                             "--sequence_parallel_enabled", "--checkpoint_dir", os.path.join(out_dir, "ckpt")])
    if rank == 0:
        torch.save((before, after), os.path.join(out_dir, f"ft_{tp}.pt"))


def _finetune_fixture(tmp_path):
    """Tiny HF Llama checkpoint + word-level tokenizer + Dolly-style JSONL (shared with the
    Lightning fine-tune test)."""
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import LlamaConfig, LlamaForCausalLM, PreTrainedTokenizerFast

    words = ("what is the color of sky grass sun water fire snow answer blue green yellow clear red white "
             "name a animal that can fly swim run bird fish horse tell me about").split()
    vocab = {w: i for i, w in enumerate(["<unk>", "<s>", "</s>", "###", "Instruction", "Context", "Answer"]
                                        + sorted(set(words)))}
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    hf_dir = str(tmp_path / "hf")
    PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>"
                            ).save_pretrained(hf_dir)
    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=64, max_position_embeddings=128, rope_theta=10000.0)
    torch.manual_seed(0)
    LlamaForCausalLM(cfg).save_pretrained(hf_dir)
    facts = [("what is the color of sky", "blue"), ("what is the color of grass", "green"),
             ("what is the color of sun", "yellow"), ("what is the color of snow", "white"),
             ("what is the color of fire", "red"), ("what is the color of water", "clear"),
             ("name a animal that can fly", "bird"), ("name a animal that can swim", "fish"),
             ("name a animal that can run", "horse")]
    data = str(tmp_path / "data.jsonl")
    with open(data, "w") as f:
        for _ in range(6):
            for q, ans in facts:
                f.write(json.dumps({"instruction": q, "context": "", "response": ans}) + "\n")
    return hf_dir, data


def test_llama_instruction_finetune_example(tmp_path):
    """examples/training/llama/tp_llama_hf_finetune.py (reference E3 fine-tuning path): HF Llama
    checkpoint + tokenizer -> TP shard -> packed Dolly-style data -> response loss drops; the
    pre-training response loss is the same at TP1 and TP2 (HF->NxD conversion + sharding)."""
    hf_dir, data = _finetune_fixture(tmp_path)
    run_distributed(_w_finetune, 2, hf_dir, data, str(tmp_path / "tp2"), 2)
    run_distributed(_w_finetune, 1, hf_dir, data, str(tmp_path / "tp1"), 1)
    b2, a2 = torch.load(tmp_path / "tp2" / "ft_2.pt")
    b1, a1 = torch.load(tmp_path / "tp1" / "ft_1.pt")
    assert abs(b1 - b2) < 1e-4 * max(1.0, abs(b1)), (b1, b2)
    assert a2 < 0.6 * b2 and a1 < 0.6 * b1, (b1, a1, b2, a2)
    assert os.path.exists(tmp_path / "tp2" / "ckpt" / "step_40" / "done")
