"""Evidence hygiene: the headline kernel-trace and PMC-traffic figures DESIGN.md quotes are the
committed profiles' own numbers -- tools/design_numbers.py prints the sentences from the latest round's files and
DESIGN.md must contain them verbatim."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _tool():
    spec = importlib.util.spec_from_file_location("design_numbers", ROOT / "tools" / "design_numbers.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_design_quotes_the_latest_committed_trace_and_traffic():
    t = _tool()
    design = (ROOT / "DESIGN.md").read_text()
    for sentence in (t.trace_sentence(), t.traffic_sentence()):
        assert sentence in design, sentence
