"""``bioengine`` command-line interface (reference bioengine/cli/cli.py:23-58).

    bioengine call <service-id> <method> [--args JSON] [--arg K=V] [--list-methods] [--json]
    bioengine apps upload|run|deploy|list|status|logs|stop ...
    bioengine cluster status

Environment: BIOENGINE_SERVER_URL, BIOENGINE_WORKER_SERVICE_ID, HYPHA_TOKEN / BIOENGINE_TOKEN.
"""
from __future__ import annotations

import click

from .. import __version__
from .apps import apps_group
from .call import call_command
from .cluster import cluster_group


@click.group()
@click.version_option(version=__version__, prog_name="bioengine")
def main():
    """BioEngine (MI355X) — deploy and call AI services on GPU workers."""


main.add_command(call_command)
main.add_command(apps_group)
main.add_command(cluster_group)
