"""Host helpers shared by the step modules (reference: grid/utils/utils.py
log :13-20, progress_bar :23-43, get_samples :76-78, setup_output_file
:92-111, open_maybe_gz :250-253).  Index/CRAM helpers are out of scope."""
from __future__ import annotations

import gzip
from contextlib import contextmanager
from pathlib import Path


def log(console, msg, style=None):
    if console:
        if style:
            console.print(msg, style=style)
        else:
            console.print(msg)
    else:
        print(msg)


class _NullProgress:
    def update(self, *a, **k):
        pass

    def advance(self, *a, **k):
        pass


@contextmanager
def progress_bar(console=None, total=1, description="Working"):
    """Rich progress bar on a console; a no-op object without one."""
    if console is None:
        yield _NullProgress(), 0
        return
    from rich.progress import BarColumn, Progress, SpinnerColumn, TaskProgressColumn, TextColumn

    with Progress(SpinnerColumn(spinner_name="dots"), TextColumn("[progress.description]{task.description}"),
                  BarColumn(), TaskProgressColumn(), console=console) as progress:
        task = progress.add_task(description, total=total)
        yield progress, task


def get_samples(samples_file):
    with open(samples_file) as f:
        return [line.strip() for line in f if line.strip()]


def setup_output_file(output_file, chrom, start, end) -> Path:
    p = Path(output_file).expanduser()
    p.parent.mkdir(parents=True, exist_ok=True)
    with open(p, "w") as f:
        f.write(f"Sample\t{chrom}:{start}-{end}\n")
    return p


def open_maybe_gz(path, mode="rt"):
    if str(path).endswith(".gz"):
        return gzip.open(path, mode)
    return open(path, mode)
