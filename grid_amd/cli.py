"""`grid` command line (reference: grid/cli.py; live command `wgs`)."""
from __future__ import annotations

import sys

import click
from rich.console import Console
from rich.theme import Theme

from . import __version__
from .utils.utils import log

grid_theme = Theme({
    "info": "#0a9396", "warning": "#ee9b00", "danger": "#9b2226", "success": "#00ff00",
    "banner": "bold #d90429", "highlight": "#94d2bd", "accent": "#ca6702",
})
console = Console(theme=grid_theme)


def print_banner():
    log(console, f"GRiD (MI355X build, grid_amd {__version__}) - Genomic Repeat inference from Depth",
        style="banner")


def _version(ctx, param, value):
    if value:
        log(console, f"GRiD version: {__version__} (grid_amd)", style="info")
        raise SystemExit(0)


@click.group(context_settings=dict(help_option_names=["-h", "--help"]))
@click.option("-v", "--version", is_flag=True, is_eager=True, expose_value=False,
              help="Show the GRiD version", callback=_version)
def cli():
    """GRiD - Genomic Repeat inference from Depth (MI355X build of steps 4-7)."""


@cli.command()
@click.argument("config", type=click.Path(exists=True))
def WGS(config):
    """Whole Genome Sequencing pipeline (steps 4-7 on the GPU)."""
    from .pipeline import run_wgs_pipeline

    print_banner()
    try:
        run_wgs_pipeline(console=console, config=config)
    except Exception as e:
        log(console, f"✗ WGS pipeline failed: {str(e)}", style="danger")
        sys.exit(1)


def main():
    try:
        cli()
    except KeyboardInterrupt:
        log(console, "\nPipeline interrupted by user", style="warning")
        sys.exit(130)
    except Exception as e:
        log(console, f"\nUnexpected error: {str(e)}", style="danger")
        sys.exit(1)


if __name__ == "__main__":
    main()
