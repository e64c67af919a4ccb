"""GPT-NeoX and BERT example models (reference examples E5 / E6): HF weights load into the TP
models, TP=1 logits/loss match HF, TP=2 (+SP for GPT-NeoX) loss and grads match TP=1."""

import torch

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps


def _neox():
    from transformers import GPTNeoXForCausalLM as HF

    from neuronx_distributed_llama3_2_amd.models.gpt_neox import gpt_neox_config

    cfg = gpt_neox_config("tiny", hidden_act="gelu")
    torch.manual_seed(0)
    return cfg, {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}


def _w_neox(rank, world, sp, out):
    from neuronx_distributed_llama3_2_amd.models.gpt_neox import GPTNeoXForCausalLM, gpt_neox_config, hf_to_nxd
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import shard_state_dict

    ps.initialize_model_parallel(world)
    cfg, sd = _neox()
    sd = hf_to_nxd(sd)
    cfg = gpt_neox_config("tiny", hidden_act="gelu", sequence_parallel_enabled=sp)
    m = GPTNeoXForCausalLM(cfg, dtype=torch.float32)
    missing, _ = m.load_state_dict(shard_state_dict(m, sd, world, rank, strict=False), strict=False)
    assert not missing, missing
    torch.manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    loss = m(ids, labels=ids).loss
    loss.backward()
    g = m.gpt_neox.layers[0].attention.query_key_value.weight.grad
    full = [torch.zeros_like(g) for _ in range(world)]
    torch.distributed.all_gather(full, g, group=ps.get_tensor_model_parallel_group())
    if rank == 0:
        torch.save({"loss": float(loss), "g": torch.cat(full)}, out)


def test_gpt_neox_matches_hf_and_tp2(tmp_path):
    from transformers import GPTNeoXForCausalLM as HF

    cfg, sd = _neox()
    hf = HF(cfg)
    hf.load_state_dict(sd)
    torch.manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        ref = float(hf(ids, labels=ids).loss)
    run_distributed(_w_neox, 1, False, str(tmp_path / "a.pt"))
    run_distributed(_w_neox, 2, True, str(tmp_path / "b.pt"))
    a, b = torch.load(tmp_path / "a.pt"), torch.load(tmp_path / "b.pt")
    assert abs(a["loss"] - ref) < 1e-4, (a["loss"], ref)
    assert abs(b["loss"] - ref) < 1e-4, (b["loss"], ref)
    assert torch.allclose(a["g"], b["g"], atol=1e-5)


def _bert():
    from transformers import BertForPreTraining as HF

    from neuronx_distributed_llama3_2_amd.models.bert import bert_config

    cfg = bert_config("tiny", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    return cfg, {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}


def _bert_batch(cfg):
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 24))
    mask = torch.ones_like(ids)
    mask[1, 18:] = 0
    tt = torch.zeros_like(ids)
    tt[:, 12:] = 1
    labels = torch.full_like(ids, -100)
    labels[:, ::5] = ids[:, ::5]
    nsp = torch.tensor([0, 1])
    return ids, mask, tt, labels, nsp


def _w_bert(rank, world, out):
    from neuronx_distributed_llama3_2_amd.models.bert import BertForPreTraining
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import shard_state_dict

    ps.initialize_model_parallel(world)
    cfg, sd = _bert()
    m = BertForPreTraining(cfg)
    missing, _ = m.load_state_dict(shard_state_dict(m, sd, world, rank, strict=False), strict=False)
    assert not [k for k in missing if "decoder" not in k], missing
    ids, mask, tt, labels, nsp = _bert_batch(cfg)
    o = m(ids, mask, tt, labels=labels, next_sentence_label=nsp)
    o.loss.backward()
    if rank == 0:
        torch.save({"loss": float(o.loss), "nsp": o.seq_relationship_logits.detach()}, out)


def test_bert_matches_hf_and_tp2(tmp_path):
    from transformers import BertForPreTraining as HF

    cfg, sd = _bert()
    hf = HF(cfg).eval()
    hf.load_state_dict(sd)
    ids, mask, tt, labels, nsp = _bert_batch(cfg)
    with torch.no_grad():
        r = hf(input_ids=ids, attention_mask=mask, token_type_ids=tt, labels=labels, next_sentence_label=nsp)
    run_distributed(_w_bert, 1, str(tmp_path / "a.pt"))
    run_distributed(_w_bert, 2, str(tmp_path / "b.pt"))
    a, b = torch.load(tmp_path / "a.pt"), torch.load(tmp_path / "b.pt")
    assert abs(a["loss"] - float(r.loss)) < 1e-4, (a["loss"], float(r.loss))
    assert abs(b["loss"] - float(r.loss)) < 1e-4
    assert torch.allclose(a["nsp"], r.seq_relationship_logits, atol=1e-4)
