from .distributed import (init_distributed_mode, cleanup, is_dist_avail_and_initialized,  # noqa: F401
                          get_world_size, get_rank, is_main_process, reduce_value, reduce_scalars,
                          barrier, get_store)
