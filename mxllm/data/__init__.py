from .datasets import CustomDataset, SyntheticTokens, imdb_like, load_text_dataset  # noqa: F401
from .tokenizer import ByteTokenizer, HFTokenizer, get_tokenizer  # noqa: F401
