from bioengine_worker_amd.utils import *  # noqa: F401,F403
from bioengine_worker_amd.utils import (create_application_from_files, create_file_list_from_directory,  # noqa: F401
                                        create_logger, check_permissions, create_context)
