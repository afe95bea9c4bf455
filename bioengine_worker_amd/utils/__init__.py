"""Cross-cutting utilities (reference: bioengine/utils/__init__.py)."""
from .artifact_utils import (create_application_from_files, create_file_list_from_directory,  # noqa: F401
                             ensure_applications_collection, get_static_site_url, validate_manifest)
from .geo_location import fetch_centroid_coordinates, fetch_geolocation  # noqa: F401
from .logger import create_logger, date_format, file_logging_format, stream_logging_format  # noqa: F401
from .network import acquire_free_port, get_internal_ip  # noqa: F401
from .permissions import check_permissions, create_context  # noqa: F401
from .requirements import get_pip_requirements, update_requirements  # noqa: F401
