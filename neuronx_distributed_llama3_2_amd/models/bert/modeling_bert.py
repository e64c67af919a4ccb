"""BERT (large) pre-training model with tensor-parallel attention and MLP
(reference: examples/training/tp_dp_bert_hf_pretrain/tp_dp_bert_large_hf_pretrain_hdf5.py:335-384,
which swaps HF BertSelfAttention / BertSelfOutput for Column/RowParallelLinear versions).

HF `BertForPreTraining` parameter names (bert.embeddings.*, bert.encoder.layer.N.attention.self.
query/key/value, attention.output.dense/LayerNorm, intermediate.dense, output.dense/LayerNorm,
bert.pooler.dense, cls.predictions.*, cls.seq_relationship) so HF checkpoints load after TP
sharding.  Beyond the reference, the FFN is tensor-parallel too.  Embeddings and the (tied) MLM
decoder are replicated, as in the reference.  Loss = masked-LM CE + next-sentence CE.
"""

from __future__ import annotations

from functools import partial
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from ...parallel_layers.layers import ColumnParallelLinear, RowParallelLinear
from ...parallel_layers.parallel_state import get_tensor_model_parallel_size
from ...parallel_layers.utils import divide
from ..attention import attention


def _init_normal(std, w):
    return nn.init.normal_(w, mean=0.0, std=std)


class BertEmbeddings(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size, padding_idx=config.pad_token_id,
                                            dtype=dtype, device=device)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size, dtype=dtype,
                                                device=device)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, config.hidden_size, dtype=dtype,
                                                  device=device)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps, dtype=dtype, device=device)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None] + \
            self.token_type_embeddings(token_type_ids)
        return self.dropout(self.LayerNorm(x))


class BertSelfAttention(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        tp = get_tensor_model_parallel_size()
        self.num_heads = config.num_attention_heads
        self.head_dim = config.hidden_size // self.num_heads
        self.heads_local = divide(self.num_heads, tp)
        init = partial(_init_normal, config.initializer_range)
        mk = partial(ColumnParallelLinear, config.hidden_size, config.hidden_size, bias=True, gather_output=False,
                     init_method=init, dtype=dtype, device=device)
        self.query, self.key, self.value = mk(), mk(), mk()
        self.dropout_p = config.attention_probs_dropout_prob

    def forward(self, x, attention_mask=None):
        B, S, _ = x.shape
        shp = (B, S, self.heads_local, self.head_dim)
        q, k, v = self.query(x).view(shp), self.key(x).view(shp), self.value(x).view(shp)
        o = attention(q, k, v, causal=False, key_padding_mask=attention_mask,
                      dropout_p=self.dropout_p if self.training else 0.0)
        return o.reshape(B, S, self.heads_local * self.head_dim)


class BertSelfOutput(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        init = partial(_init_normal, config.initializer_range)
        self.dense = RowParallelLinear(config.hidden_size, config.hidden_size, bias=True, input_is_parallel=True,
                                       init_method=init, dtype=dtype, device=device)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps, dtype=dtype, device=device)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, h, x):
        return self.LayerNorm(self.dropout(self.dense(h)) + x)


class BertAttention(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.self = BertSelfAttention(config, dtype, device)
        self.output = BertSelfOutput(config, dtype, device)

    def forward(self, x, attention_mask=None):
        return self.output(self.self(x, attention_mask), x)


class BertIntermediate(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        init = partial(_init_normal, config.initializer_range)
        self.dense = ColumnParallelLinear(config.hidden_size, config.intermediate_size, bias=True, gather_output=False,
                                          init_method=init, dtype=dtype, device=device)
        from transformers.activations import ACT2FN

        self.act = ACT2FN[config.hidden_act]

    def forward(self, x):
        return self.act(self.dense(x))


class BertOutput(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        init = partial(_init_normal, config.initializer_range)
        self.dense = RowParallelLinear(config.intermediate_size, config.hidden_size, bias=True, input_is_parallel=True,
                                       init_method=init, dtype=dtype, device=device)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps, dtype=dtype, device=device)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, h, x):
        return self.LayerNorm(self.dropout(self.dense(h)) + x)


class BertLayer(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.attention = BertAttention(config, dtype, device)
        self.intermediate = BertIntermediate(config, dtype, device)
        self.output = BertOutput(config, dtype, device)

    def forward(self, x, attention_mask=None):
        a = self.attention(x, attention_mask)
        return self.output(self.intermediate(a), a)


class BertEncoder(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(config, dtype, device) for _ in range(config.num_hidden_layers)])

    def forward(self, x, attention_mask=None):
        for layer in self.layer:
            x = layer(x, attention_mask)
        return x


class BertPooler(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size, dtype=dtype, device=device)

    def forward(self, x):
        return torch.tanh(self.dense(x[:, 0]))


class BertModel(nn.Module):
    def __init__(self, config, dtype=torch.float32, device=None):
        super().__init__()
        self.embeddings = BertEmbeddings(config, dtype, device)
        self.encoder = BertEncoder(config, dtype, device)
        self.pooler = BertPooler(config, dtype, device)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None):
        x = self.encoder(self.embeddings(input_ids, token_type_ids), attention_mask)
        return x, self.pooler(x)


class BertPredictionHeadTransform(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        from transformers.activations import ACT2FN

        self.dense = nn.Linear(config.hidden_size, config.hidden_size, dtype=dtype, device=device)
        self.act = ACT2FN[config.hidden_act]
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps, dtype=dtype, device=device)

    def forward(self, x):
        return self.LayerNorm(self.act(self.dense(x)))


class BertLMPredictionHead(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.transform = BertPredictionHeadTransform(config, dtype, device)
        self.decoder = nn.Linear(config.hidden_size, config.vocab_size, bias=False, dtype=dtype, device=device)
        self.bias = nn.Parameter(torch.zeros(config.vocab_size, dtype=dtype, device=device))

    def forward(self, x):
        return self.decoder(self.transform(x)) + self.bias


class BertPreTrainingHeads(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, dtype, device)
        self.seq_relationship = nn.Linear(config.hidden_size, 2, dtype=dtype, device=device)

    def forward(self, seq, pooled):
        return self.predictions(seq), self.seq_relationship(pooled)


class BertPreTrainingOutput(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class BertForPreTraining(nn.Module):
    def __init__(self, config, dtype=torch.float32, device=None):
        super().__init__()
        self.config = config
        self.bert = BertModel(config, dtype, device)
        self.cls = BertPreTrainingHeads(config, dtype, device)
        self.cls.predictions.decoder.weight = self.bert.embeddings.word_embeddings.weight   # tied

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None, next_sentence_label=None,
                **unused):
        seq, pooled = self.bert(input_ids, attention_mask, token_type_ids)
        mlm, nsp = self.cls(seq, pooled)
        loss = None
        if labels is not None:
            loss = F.cross_entropy(mlm.float().view(-1, mlm.shape[-1]), labels.view(-1), ignore_index=-100)
            if next_sentence_label is not None:
                loss = loss + F.cross_entropy(nsp.float(), next_sentence_label.view(-1))
        return BertPreTrainingOutput(loss=loss, prediction_logits=mlm, seq_relationship_logits=nsp)


def bert_config(name: str = "bert-large-uncased", **overrides):
    from transformers import BertConfig

    presets = {
        "bert-large-uncased": dict(vocab_size=30522, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                   intermediate_size=4096, max_position_embeddings=512, type_vocab_size=2),
        "tiny": dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=256, max_position_embeddings=128, type_vocab_size=2),
    }
    kw = dict(presets[name])
    kw.update(overrides)
    return BertConfig(**kw)
