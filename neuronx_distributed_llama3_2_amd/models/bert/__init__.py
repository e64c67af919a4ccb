from .modeling_bert import BertForPreTraining, BertModel, bert_config  # noqa: F401
