"""The K2 end-game answer applied in one pass (md_env.h env_endgame_apply) rests on a closed
form: in a state of pairs joined in both layers plus isolated nodes, covering a node of a pair
kills its two edges and isolates its partner, nothing is pruned, and the LMCC after action j
(U/Mcc.py:30-38, over non-covered nodes) is 2 while pairs remain, else 1 while a non-covered
node remains, else 0; the loop stops after the action that takes the last pair
(U/mvc_env.py:74-87, isTerminal :128-131).  Checked here against the oracle environment stepped
action by action on random end-game states -- including picks of isolated nodes and of a node
whose partner was picked earlier, and answers longer than the terminal cut."""
import random

import numpy as np

from oracle import refenv


def closed_form(n, pairs, actions):
    """(applied actions, LMCC after each) by env_endgame_apply's rule."""
    part = {}
    for u, v in pairs:
        part[u], part[v] = v, u
    left, picked, out = len(pairs), set(), []
    for j, a in enumerate(actions):
        if left == 0:
            break  # terminal before this action
        b = part.get(a)
        if b is not None and b not in picked:
            left -= 1
        picked.add(a)
        out.append(2 if left > 0 else (1 if n - (j + 1) > 0 else 0))
    return out


def test_endgame_closed_form_matches_oracle():
    rng = random.Random(7)
    for _ in range(60):
        n = rng.randint(2, 40)
        nodes = list(range(n))
        rng.shuffle(nodes)
        npairs = rng.randint(1, n // 2)
        pairs = [(nodes[2 * i], nodes[2 * i + 1]) for i in range(npairs)]
        e = np.array(pairs, np.int32)
        # layer 1 lists the same pairs in another order and orientation
        e1 = np.array([(v, u) if rng.random() < 0.5 else (u, v) for u, v in rng.sample(pairs, len(pairs))], np.int32)
        g = refenv.RefGraph(n, e, e1)
        env = refenv.RefEnv(g, "unit")
        actions = rng.sample(range(n), rng.randint(1, n))
        want = closed_form(n, pairs, actions)
        got = []
        for a in actions:
            if env.terminal():
                break
            got.append(env.step(int(a)))
        assert got == want, (n, pairs, actions)
        assert env.terminal() == (got[-1] != 2)  # terminal once no pair is left
