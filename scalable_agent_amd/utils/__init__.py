from .utils import (AttrDict, str2bool, log, ensure_dir_exists, project_root,
                    experiment_dir, cfg_file, memory_consumption_mb)
from . import nest
