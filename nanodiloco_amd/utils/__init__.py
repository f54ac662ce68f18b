from .seed import set_seed_all, rank_seed
from .run_name import create_run_name
from .schedule import cosine_with_warmup, CosineWarmupSchedule

__all__ = ["set_seed_all", "rank_seed", "create_run_name", "cosine_with_warmup", "CosineWarmupSchedule"]
