"""``python main.py [development|staging|production] [options]`` — see k8s_watcher_amd/cli.py."""

from k8s_watcher_amd.cli import entrypoint

if __name__ == "__main__":
    entrypoint()
