"""Where autograd adds gradients in the OC2 optimizer step: the backward graph's (node, input)
slots that receive gradient from more than one consumer (each extra one is an elementwise add
launch on the GPU). CPU, on the oc2_update fixture; prints slots by gradient size.

    python tools/oc2_grad_fanin.py [fixture]
"""

import collections
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "swarmacb-isaaclab_amd")

import torch  # noqa: E402

import oc2_fixtures as O2  # noqa: E402


def main(name="oc2_update"):
    tr, fx, _names, _named = O2.make_oc2_trainer(name, "cpu", False)
    O2.load_buffer(tr, fx)
    captured = {}
    orig = tr.compute_losses

    def grab(batch, eps, ref=None):
        out = orig(batch, eps, ref)
        if not captured:
            captured["losses"] = out
        raise StopIteration

    tr.compute_losses = grab
    epochs = O2.oracle_batches_per_epoch(tr, fx)
    tr._sequence_batches = lambda: iter(epochs.pop(0))
    try:
        tr.update()
    except StopIteration:
        pass
    _terms, actor_loss, critic_loss = tr.objectives(captured["losses"])
    for tag, loss in (("actor", actor_loss), ("critic", critic_loss)):
        refs = collections.Counter()
        seen, stack = set(), [loss.grad_fn]
        while stack:
            n = stack.pop()
            if n is None or n in seen:
                continue
            seen.add(n)
            for nxt, slot in n.next_functions:
                if nxt is not None:
                    refs[(nxt, slot)] += 1
                    stack.append(nxt)
        fan = [(k, c) for k, c in refs.items() if c > 1]
        rows = []
        for (node, slot), c in fan:
            shape = tuple(node.variable.shape) if hasattr(node, "variable") else None
            if shape is None:
                meta = getattr(node, "_input_metadata", None)
                shape = meta[slot].shape if meta else "?"
            rows.append((c - 1, node.name(), slot, shape))
        print(f"{tag}: {len(seen)} nodes, {sum(r[0] for r in rows)} gradient adds")
        for extra, nm, slot, shape in sorted(rows, key=lambda r: str(r[3])):
            print(f"  +{extra}  {nm}[{slot}]  {shape}")


if __name__ == "__main__":
    main(*sys.argv[1:])
