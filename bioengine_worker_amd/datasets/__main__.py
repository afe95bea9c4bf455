"""``python -m bioengine_worker_amd.datasets --data-dir PATH`` (reference: bioengine/datasets/__main__.py)."""
import argparse

from .server import start_proxy_server


def main(argv=None):
    ap = argparse.ArgumentParser(description="BioEngine Datasets - privacy-preserving dataset streaming server")
    ap.add_argument("--data-dir", required=True, help="directory of dataset subdirectories with manifest.yaml")
    ap.add_argument("--server-ip", default=None)
    ap.add_argument("--server-port", type=int, default=None)
    ap.add_argument("--authentication-server-url", default=None,
                    help="hub/Hypha used to validate tokens (local://name, ws://host:port, https://...)")
    ap.add_argument("--log-file", default=None)
    a = ap.parse_args(argv)
    start_proxy_server(a.data_dir, a.server_ip, a.server_port, a.authentication_server_url, a.log_file)


if __name__ == "__main__":
    main()
