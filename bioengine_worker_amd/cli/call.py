"""``bioengine call SERVICE [METHOD] [--args JSON] [--arg K=V ...] [--list-methods] [--json]``
(reference bioengine/cli/call.py:48-184)."""
from __future__ import annotations

import json
import sys

import click

from . import common


@click.command("call")
@click.argument("service_id")
@click.argument("method", required=False)
@click.option("--args", "args_json", default=None, metavar="JSON", help="Arguments as a JSON object.")
@click.option("--arg", "pairs", multiple=True, metavar="KEY=VALUE", help="One argument (auto-typed); repeatable.")
@click.option("--list-methods", is_flag=True, help="List the service's methods.")
@click.option("--json", "as_json", is_flag=True, help="JSON output (default when stdout is not a TTY).")
@click.option("--token", default=None, help="Auth token (env HYPHA_TOKEN / BIOENGINE_TOKEN).")
@click.option("--server-url", default=None, hidden=True)
def call_command(service_id, method, args_json, pairs, list_methods, as_json, token, server_url):
    """Call METHOD of any deployed service SERVICE_ID."""
    want_json = as_json or not sys.stdout.isatty()

    async def go():
        try:
            srv, svc = await common.get_service(common.server_url(server_url), service_id, common.token(token))
        except Exception as e:  # noqa: BLE001
            common.fail(f"could not connect to service '{service_id}': {e}", "check the id and that it is running")
        if list_methods:
            names = common.method_names(svc)
            if want_json:
                common.print_json({"service_id": service_id, "methods": names})
            else:
                click.echo(f"Methods of '{service_id}':")
                for n in names:
                    click.echo(f"  {n}")
            return
        if not method:
            common.fail("no method given", "pass a method name or --list-methods")
        kwargs = {}
        if args_json:
            try:
                kwargs = json.loads(args_json)
            except json.JSONDecodeError as e:
                common.fail(f"--args is not valid JSON: {e}")
        for kv in pairs:
            if "=" not in kv:
                common.fail(f"--arg '{kv}' must be KEY=VALUE")
            k, v = kv.split("=", 1)
            kwargs[k] = common.parse_value(v)
        fn = getattr(svc, method, None)
        if fn is None:
            common.fail(f"service '{service_id}' has no method '{method}'", "use --list-methods")
        try:
            res = await fn(**kwargs)
        except Exception as e:  # noqa: BLE001
            common.fail(f"call to '{method}' failed: {e}")
        if want_json or isinstance(res, (dict, list)):
            common.print_json(res)
        else:
            click.echo(str(res))

    common.run(go())
