"""ORACLE (test infrastructure only) -- pure-Python restatement of the reference's batched
self-play search: PUCT evaluator, coroutine leaf-batching scheduler, self-play driver, pool
manager, inline Supervisor and Player.

Follows (reference file:line):
  PuctNode::create / reply             src/cpp/puct/node.cpp:153-221, 463-511
  sorts                                node.cpp:316-373, evaluator.cpp:242-279
  PuctEvaluator                        src/cpp/puct/evaluator.cpp:165-1510
  NetworkScheduler                     src/cpp/scheduler.cpp:70-241
  SelfPlay                             src/cpp/selfplay.cpp:43-343
  SelfPlayManager / UniqueStates       src/cpp/selfplaymanager.cpp:72-159, uniquestates.h:28-76
  Supervisor (inline) / Player         src/cpp/supervisor.cpp:101-127, player.cpp:16-173

Greenlets are Python generators (``yield from`` along the call chain that can reach evaluate()).
C float arithmetic is emulated with numpy.float32 scalars (F32) and C double with Python floats,
expression by expression as the C++ is written (no FMA contraction); std::sort, libm and the RNG
come from oracle/stdlib_ref.py.  Only small cases run here (pure-Python loops).
"""
from collections import deque

import numpy as np

from . import stdlib_ref as S

F32 = np.float32
FLT_MIN = float(np.finfo(np.float32).tiny)


class Child(object):
    __slots__ = ("to_node", "unselectable", "traversals", "policy_prob_orig", "policy_prob", "next_prob",
                 "debug_node_score", "debug_puct_score", "move")

    def __init__(self, move):
        self.to_node = None
        self.unselectable = False
        self.traversals = 0
        self.policy_prob_orig = F32(1.0)
        self.policy_prob = F32(1.0)
        self.next_prob = F32(0.0)
        self.debug_node_score = F32(0.0)
        self.debug_puct_score = F32(0.0)
        self.move = move


class Node(object):
    def __init__(self):
        self.parent = None
        self.visits = 0
        self.inflight_visits = 0
        self.ref_count = 1
        self.unselectable_count = 0
        self.num_children = 0
        self.num_children_expanded = 0
        self.puct_constant = F32(1.44)
        self.is_finalised = False
        self.force_terminal = False
        self.dirichlet_noise_set = False
        self.lead_role_index = 0
        self.game_depth = 0
        self.current = []
        self.final = []
        self.state = 0
        self.children = []

    def is_terminal(self):
        return self.force_terminal or self.num_children == 0

    def final_clamped(self, ri):
        s = self.final[ri]
        return F32(0.0) if s < F32(0.0) else (F32(1.0) if s > F32(1.0) else s)

    def normaliseX(self):
        total = F32(0)
        for c in self.children:
            total = F32(total + c.policy_prob)
        if float(total) > FLT_MIN:
            for c in self.children:
                c.policy_prob = F32(c.policy_prob / total)
        else:
            for c in self.children:
                c.policy_prob = F32(1.0 / self.num_children)


def node_create(state, sm):
    """node.cpp:153-221 (children = cross product of legal moves, role 0 outermost)."""
    rc = sm.role_count
    node = Node()
    node.state = state
    lead = 0
    finalised = True
    legals = None
    if not sm.is_terminal(state):
        finalised = False
        legals = [sm.legal(state, r) for r in range(rc)]
        maxm = 1
        for r in range(rc):
            if len(legals[r]) > maxm:
                maxm = len(legals[r])
                lead = r
        if maxm > 1:
            if any(r != lead and len(legals[r]) > 1 for r in range(rc)):
                lead = -1
    node.lead_role_index = lead
    node.is_finalised = finalised
    node.current = [F32(0.0)] * rc
    node.final = [F32(0.0)] * rc
    if not finalised:
        moves = [()]
        for r in range(rc):
            moves = [m + (a,) for m in moves for a in legals[r]]
        node.children = [Child(m) for m in moves]
        node.num_children = len(node.children)
    else:
        for r in range(rc):
            v = F32(sm.goal(state, r) / 100.0)
            node.final[r] = v
            node.current[r] = v
    return node


def sorted_children(node, next_probability=False):
    """node.cpp:316-343"""
    def less(a, b):
        va = a.to_node.visits if a.to_node is not None else 0
        vb = b.to_node.visits if b.to_node is not None else 0
        if va == vb:
            return a.next_prob > b.next_prob if next_probability else a.policy_prob > b.policy_prob
        return va > vb
    return S.std_sort(list(node.children), less)


def sorted_children_traversals(node, next_probability=False):
    """node.cpp:346-373"""
    def less(a, b):
        if a.traversals == b.traversals:
            return a.next_prob > b.next_prob if next_probability else a.policy_prob > b.policy_prob
        return a.traversals > b.traversals
    return S.std_sort(list(node.children), less)


def sorted_children_select(node):
    """evaluator.cpp:242-263"""
    lead = node.lead_role_index

    def less(a, b):
        sa = a.to_node.current[lead] if a.to_node is not None else F32(-1)
        sb = b.to_node.current[lead] if b.to_node is not None else F32(-1)
        if sa < 0 and sb < 0:
            return a.policy_prob_orig > b.policy_prob_orig
        return sa > sb
    return S.std_sort(list(node.children), less)


class Request(object):
    def __init__(self, node):
        self.node = node


class Evaluator(object):
    def __init__(self, sm, scheduler, planes, num_rewards):
        self.sm = sm
        self.scheduler = scheduler
        self.planes = planes
        self.num_rewards = num_rewards
        self.conf = None
        self.game_depth = 0
        self.initial_root = None
        self.root = None
        self.number_of_nodes = 0
        self.do_playouts = False
        self.rng = S.Rng()
        self.stats = {}
        self.reset_stats()

    def reset_stats(self):
        self.stats = dict(num_blocked=0, num_tree_playouts=0, num_evaluations=0, playouts_finals=0)

    def update_conf(self, conf):
        self.conf = conf

    # ---- tree management (evaluator.cpp:102-239) ------------------------------------------
    def release_nodes(self, current, garbage):
        for c in current.children:
            if c.to_node is not None:
                nxt = c.to_node
                if nxt.ref_count <= 0:
                    continue
                c.to_node = None
                nxt.ref_count -= 1
                if nxt.ref_count == 0:
                    self.release_nodes(nxt, garbage)
                    garbage.append(nxt)

    def create_node(self, parent, state):
        node = node_create(state, self.sm)
        self.number_of_nodes += 1
        node.parent = parent
        if parent is not None:
            node.game_depth = parent.game_depth + 1
            parent.num_children_expanded += 1
        else:
            node.game_depth = self.game_depth
        if node.is_finalised:
            for ii in range(self.sm.role_count):
                s = node.current[ii]
                if float(s) > 0.99:
                    node.current[ii] = F32(float(s) * 1.05)
                elif float(s) < 0.01:
                    node.current[ii] = F32(-0.05)
            return node
        if node.num_children == 1:
            return node
        yield from self.scheduler.evaluate(self, node)
        self.stats["num_evaluations"] += 1
        return node

    def reply(self, node, policies, rewards):
        """node.cpp:463-511"""
        rc = len(policies)
        raw = policies[node.lead_role_index]
        total = F32(0.0)
        for c in node.children:
            x = F32(raw[c.move[node.lead_role_index]])
            c.policy_prob_orig = x if F32(0.001) < x else F32(0.001)
            total = F32(total + c.policy_prob_orig)
        for c in node.children:
            c.policy_prob_orig = F32(c.policy_prob_orig / total)
            c.policy_prob = c.policy_prob_orig
        for ri in range(rc):
            s = F32(rewards[ri])
            if self.num_rewards == 3:
                mid = F32(F32(rewards[2]) / F32(2.0))
                s = F32(s + mid)
            if float(s) > 1.0:
                s = F32(1.0)
            elif float(s) < 0.0:
                s = F32(0.0)
            node.final[ri] = s
            node.current[ri] = node.final_clamped(ri)

    def expand_child(self, parent, child):
        state = self.sm.next_state(parent.state, child.move)
        child.unselectable = True
        parent.unselectable_count += 1
        child.to_node = yield from self.create_node(parent, state)
        parent.unselectable_count -= 1
        child.unselectable = False
        return child.to_node

    # ---- selection (evaluator.cpp:341-517) ------------------------------------------------
    def select_child(self, node, path):
        assert not node.is_terminal()
        depth = len(path)
        self.set_puct_constant(node, depth)
        if node.num_children == 1:
            c = node.children[0]
            path.append((node, c, c))
            return c
        if depth == 0:
            self.set_dirichlet_noise(node)
        prior_score = self.prior_score(node, depth)
        sqrt_node_visits = float(np.sqrt(float(node.visits + 1)))
        best_score = F32(-1)
        best_child = None
        best_child_score_actual_score = F32(-1)
        best_child_score = None
        bad_fallback = None
        best_fallback_score = F32(-1)
        best_fallback = None
        unselectables = 0
        lead = node.lead_role_index
        for c in sorted_children_select(node):
            if c.unselectable:
                unselectables += 1
                continue
            elif c.to_node is not None and (c.to_node.num_children > 0 and
                                            c.to_node.unselectable_count == c.to_node.num_children):
                unselectables += 1
                continue
            child_score = float(prior_score)
            traversals = c.traversals + 1
            inflight = float(c.to_node.inflight_visits) if c.to_node is not None else 0.0
            exploration = float(F32(node.puct_constant * c.policy_prob)) * sqrt_node_visits / (traversals + inflight)
            if c.to_node is not None:
                cn = c.to_node
                child_score = float(cn.current[lead])
                if cn.is_finalised:
                    if child_score > 0.99:
                        if depth > 0:
                            path.append((node, c, c))
                            return c
                        child_score = child_score * float(F32(F32(1.0) + node.puct_constant))
                    elif child_score < 0.01:
                        bad_fallback = c
                        continue
                    else:
                        exploration = 0.0
                if (cn.is_finalised or cn.visits > 42) and child_score > float(best_child_score_actual_score):
                    best_child_score_actual_score = F32(child_score)
                    best_child_score = c
            if c.traversals > 0 and inflight > 0:
                discounted = inflight * (self.rng.get() + 0.5)
                child_score = (child_score * c.traversals) / (c.traversals + discounted)
            limit_latch_root = F32(0.66)
            c.debug_node_score = F32(child_score)
            c.debug_puct_score = F32(exploration)
            score = child_score + exploration
            if node.visits > 1000 and node.visits < 40000000 and depth == 0 and self.rng.get() > 0.1:
                if c.traversals > 16 and F32(c.traversals) > F32(F32(node.visits) * limit_latch_root):
                    if best_fallback is None or score > float(best_fallback_score):
                        best_fallback = c
                        best_fallback_score = F32(score)
                    continue
            if score > float(best_score):
                best_child = c
                best_score = F32(score)
        if best_child is None:
            if best_fallback is not None:
                best_child = best_child_score if best_child_score is not None else best_fallback
            elif bad_fallback is not None:
                if unselectables > 0:
                    yield from self.scheduler.yield_()
                best_child = bad_fallback
            else:
                self.stats["num_blocked"] += 1
        if best_child_score is None:
            best_child_score = best_child
        if best_child is not None:
            path.append((node, best_child, best_child_score))
        return best_child

    # ---- backup (evaluator.cpp:519-656) ---------------------------------------------------
    def backup(self, new_scores, path):
        rc = self.sm.role_count
        bp_once = bool(self.conf["backup_finalised"])
        for index in range(len(path) - 1, -1, -1):
            node, choice, _ = path[index]
            if bp_once and not node.is_finalised and node.lead_role_index >= 0:
                bp_once = False
                fc = self._force_finalise(node)
                if fc is not None:
                    for ii in range(rc):
                        node.current[ii] = fc.to_node.current[ii]
                    node.is_finalised = True
            if node.is_finalised:
                for ii in range(rc):
                    new_scores[ii] = node.current[ii]
            else:
                for ii in range(rc):
                    visits = F32(node.visits)
                    if visits > F32(100000):
                        visits = F32(F32(100000) + F32(F32(0.1) * F32(visits - F32(100000))))
                    node.current[ii] = F32(F32(F32(visits * node.current[ii]) + new_scores[ii]) /
                                           F32(visits + F32(1.0)))
            node.visits += 1
            if node.inflight_visits > 0:
                node.inflight_visits -= 1
            if choice is not None:
                choice.traversals += 1
                if node.visits > 23:
                    cur = float(node.current[node.lead_role_index])
                    if cur > 0.3 and cur < 0.7:
                        apply, minimum = F32(0.995), F32(0.02)
                    elif cur > 0.15 and cur < 0.85:
                        apply, minimum = F32(0.9975), F32(0.03)
                    else:
                        apply, minimum = F32(0.9975), F32(0.10)
                    if choice.policy_prob > minimum:
                        choice.policy_prob = F32(choice.policy_prob * apply)
                        choice.policy_prob = choice.policy_prob if minimum < choice.policy_prob else minimum
            if node.visits % 100 == 0:
                node.normaliseX()

    def _force_finalise(self, cur):
        best_score, best, more = F32(-1), None, False
        for c in cur.children:
            if c.to_node is not None and c.to_node.is_finalised:
                score = c.to_node.current[cur.lead_role_index]
                if float(score) > 0.99:
                    return c
                if score > best_score:
                    best_score, best = score, c
            else:
                more = True
        return None if more else best

    # ---- playouts (evaluator.cpp:658-886) ---------------------------------------------------
    def tree_playout(self, current, path):
        assert current is not None and not current.is_terminal()
        while True:
            if current.is_terminal() or current.is_finalised:
                path.append((current, None, None))
                break
            while True:
                child = yield from self.select_child(current, path)
                if child is not None:
                    break
                yield from self.scheduler.yield_()
            if child.to_node is None:
                current = yield from self.expand_child(current, child)
                if current.is_finalised or current.num_children > 1:
                    path.append((current, None, None))
                    break
            current.inflight_visits += 1
            current = child.to_node
        if current.is_finalised:
            self.stats["playouts_finals"] += 1
        scores = [current.current[ii] for ii in range(self.sm.role_count)]
        self.backup(scores, path)
        self.stats["num_tree_playouts"] += 1
        return len(path)

    def playout_worker(self, counter):
        while self.do_playouts:
            if self.stats["num_tree_playouts"] % 10000 == 0:
                yield from self.scheduler.yield_()
            if self.root.is_finalised:
                break
            yield from self.tree_playout(self.root, [])
        counter[0] -= 1

    def playout_main(self, max_evaluations):
        conf = self.conf
        # int * float -> float, truncated back to int (evaluator.cpp:782)
        max_non_converged = int(F32(F32(max_evaluations) * F32(conf["evaluation_multiplier_to_convergence"])))
        max_tree_playouts = 4 * max_non_converged
        # build extension spin_yield_playouts (engine/config.h, evaluator.cpp playoutMain): yield
        # the coroutine after that many consecutive NN-free playouts; 0 = the reference's loop
        spin = int(conf.get("spin_yield_playouts", 0) or 0)
        evals_seen, quiet = self.stats["num_evaluations"], 0
        while True:
            is_converged = self.converged(conf["converged_visits"])
            if self.root.is_finalised and self.stats["num_tree_playouts"] > 100:
                break
            if is_converged and self.stats["num_tree_playouts"] > max_tree_playouts:
                break
            if self.number_of_nodes > 50000000:
                break
            if is_converged and self.stats["num_evaluations"] > max_evaluations:
                break
            if not is_converged and self.stats["num_evaluations"] > max_non_converged:
                break
            yield from self.tree_playout(self.root, [])
            if spin > 0:
                if self.stats["num_evaluations"] != evals_seen:
                    evals_seen, quiet = self.stats["num_evaluations"], 0
                else:
                    quiet += 1
                    if quiet >= spin:
                        quiet = 0
                        yield from self.scheduler.yield_()

    # ---- moves (evaluator.cpp:888-1098) -----------------------------------------------------
    def fast_apply_move(self, nxt):
        new_root = None
        garbage = []
        for c in self.root.children:
            if c is nxt:
                if c.to_node is None:
                    yield from self.expand_child(self.root, c)
                new_root = c.to_node
            elif c.to_node is not None:
                n = c.to_node
                c.to_node = None
                n.ref_count -= 1
                if n.ref_count == 0:
                    self.release_nodes(n, garbage)
                    garbage.append(n)
        self.number_of_nodes -= len(garbage)
        self.root = new_root
        self.game_depth += 1
        return self.root

    def apply_move(self, move):
        for c in self.root.children:
            if tuple(c.move) == tuple(move):
                yield from self.fast_apply_move(c)
                break

    def reset(self, game_depth):
        if self.initial_root is not None:
            garbage = []
            self.release_nodes(self.initial_root, garbage)
            garbage.append(self.initial_root)
            self.number_of_nodes -= len(garbage)
            self.initial_root = self.root = None
        self.reset_stats()
        self.game_depth = game_depth

    def establish_root(self, state):
        if state is None:
            state = self.sm.initial_state
        self.root = yield from self.create_node(None, state)
        self.initial_root = self.root
        return self.root

    def reset_root_node(self):
        for c in self.root.children:
            c.policy_prob = c.policy_prob_orig
            c.traversals = min(1, c.traversals)
        self.root.dirichlet_noise_set = False

    def on_next_move(self, max_evaluations):
        self.reset_stats()
        self.do_playouts = True
        conf = self.conf
        if float(F32(conf["think_time"])) > 10 and not self.root.dirichlet_noise_set and \
                not self.root.is_finalised and self.root.visits > 10000:
            if self.number_of_nodes < 3000000:
                self.reset_root_node()
        counter = [0]
        if conf["batch_size"] > 1 and self.root is not None and not self.root.is_finalised:
            if max_evaluations < 0 or max_evaluations > 100:
                for _ in range(conf["batch_size"] - 1):
                    counter[0] += 1
                    self.scheduler.add_runnable(self.playout_worker(counter))
        if max_evaluations != 0:
            yield from self.playout_main(max_evaluations)
        self.do_playouts = False
        while counter[0] > 0:
            yield from self.scheduler.yield_()
        return self.choose(self.root)

    # ---- choices (evaluator.cpp:1100-1510) --------------------------------------------------
    def choose_top_visits(self, node):
        children = sorted_children_traversals(node)
        ri = node.lead_role_index
        indx0 = indx1 = -1
        count = 0
        for c in children:
            if c.to_node is not None and c.to_node.is_finalised:
                if float(c.to_node.current[ri]) > 0.99:
                    return c
                if float(c.to_node.current[ri]) < 0.01:
                    count += 1
                    continue
            if indx0 == -1:
                indx0 = count
            elif indx1 == -1:
                indx1 = count
            count += 1
        ratio = F32(self.conf["top_visits_best_guess_converge_ratio"])
        if ratio > 0 and indx0 != -1 and indx1 != -1:
            c0, c1 = children[indx0], children[indx1]
            if c0.to_node is not None and c1.to_node is not None:
                if F32(c1.traversals) > F32(F32(c0.traversals) * ratio) and c1.to_node.current[ri] > c0.to_node.current[ri]:
                    return c1
                return c0
        return children[0]

    def get_probabilities(self, node, temperature, use_policy):
        node_visits = F32(node.visits + 0.001 * node.num_children)
        total = F32(0.0)
        for c in node.children:
            child_visits = F32(F32(c.traversals) + F32(0.001)) if c.to_node is not None else F32(0.001)
            if use_policy:
                c.next_prob = F32(c.policy_prob + F32(0.001))
            else:
                c.next_prob = F32(child_visits / node_visits)
            c.next_prob = F32(S.pow_d(float(c.next_prob), float(temperature)))
            total = F32(total + c.next_prob)
        for c in node.children:
            c.next_prob = F32(c.next_prob / total)
        return sorted_children(node, True)

    def prior_score(self, node, depth):
        prior = node.final[node.lead_role_index]
        if node.visits > 8:
            best = self.choose_top_visits(node)
            if best.to_node is not None:
                prior = best.to_node.current[node.lead_role_index]
        fpu = F32(self.conf["fpu_prior_discount_root"] if depth == 0 else self.conf["fpu_prior_discount"])
        if fpu > 0:
            total = F32(0.0)
            for c in node.children:
                if c.to_node is not None and c.to_node.visits > 0:
                    total = F32(total + c.policy_prob)
            fpu = F32(fpu * S.sqrtf(total))
            prior = F32(prior - fpu)
        return prior

    def set_dirichlet_noise(self, node):
        pct = F32(self.conf["dirichlet_noise_pct"])
        if node.dirichlet_noise_set or node.num_children < 2 or pct < 0:
            return
        if float(node.current[node.lead_role_index]) > 0.95:
            return
        alpha = F32(F32(10.83) / F32(node.num_children))
        gamma = S.GammaF32(alpha, 1.0)
        noise = []
        total = F32(0.0)
        for _ in range(node.num_children):
            x = gamma(self.rng)
            noise.append(x)
            total = F32(total + x)
        if float(total) < FLT_MIN:
            return
        noise = [F32(x / total) for x in noise]
        squash_pct = F32(self.conf["noise_policy_squash_pct"])
        squash = squash_pct > 0 and self.rng.get() < float(squash_pct)
        squash_prob = F32(self.conf["noise_policy_squash_prob"])
        tp = F32(0.0)
        for c, nz in zip(node.children, noise):
            if squash:
                c.policy_prob = c.policy_prob if c.policy_prob < squash_prob else squash_prob
            c.policy_prob = F32(F32(F32(F32(1.0) - pct) * c.policy_prob) + F32(pct * nz))
            tp = F32(tp + c.policy_prob)
        for c in node.children:
            c.policy_prob = F32(c.policy_prob / tp)
        node.dirichlet_noise_set = True

    def set_puct_constant(self, node, depth):
        base = F32(19652.0)
        pc = F32(self.conf["puct_constant_root"] if depth == 0 else self.conf["puct_constant"])
        node.puct_constant = S.logf(F32(F32(F32(1 + node.visits) + base) / base))
        node.puct_constant = F32(node.puct_constant + pc)

    def get_temperature(self, depth):
        conf = self.conf
        if depth >= conf["depth_temperature_stop"]:
            return F32(-1)
        mult = F32(F32(1.0) + F32(F32(depth - conf["depth_temperature_start"]) * F32(conf["depth_temperature_increment"])))
        mult = mult if F32(1.0) < mult else F32(1.0)
        t = F32(F32(conf["temperature"]) * mult)
        mx = F32(conf["depth_temperature_max"])
        return mx if mx < t else t

    def choose(self, node):
        if self.conf["choose"] == "choose_temperature":
            return self.choose_temperature(node)
        return self.choose_top_visits(node)

    def converged(self, count):
        children = sorted_children(self.root)
        if len(children) >= 2:
            n0, n1 = children[0].to_node, children[1].to_node
            if n0 is not None and n1 is not None:
                ri = self.root.lead_role_index
                if n0.current[ri] > n1.current[ri] and n0.visits > n1.visits + count:
                    return True
            return False
        return True

    def choose_temperature(self, node):
        temperature = self.get_temperature(node.game_depth)
        if temperature < 0:
            return self.choose_top_visits(node)
        if float(F32(self.conf["dirichlet_noise_pct"])) < 0 and node.visits < 3:
            dist = self.get_probabilities(self.root, temperature, True)
        else:
            dist = self.get_probabilities(self.root, temperature, False)
        expected = F32(self.rng.get() * float(F32(self.conf["random_scale"])))
        seen = F32(0)
        for c in dist:
            seen = F32(seen + c.next_prob)
            if seen > expected:
                return c
        return dist[-1]


class Scheduler(object):
    """scheduler.cpp:70-241 with generators as coroutines."""

    def __init__(self, planes, batch_size, num_prev_states, policy_sizes, num_rewards):
        self.planes = planes
        self.batch_size = batch_size
        self.num_prev_states = num_prev_states
        self.policy_sizes = policy_sizes
        self.num_rewards = num_rewards
        self.requestors = []
        self.yielders = []
        self.runnables = deque()
        self.main = None
        self.buf = []
        self.pde = None

    def evaluate(self, evaluator, node):
        prev, cur = [], node.parent
        for _ in range(self.num_prev_states):
            if cur is not None:
                prev.append(cur.state)
                cur = cur.parent
        self.buf.append(self.planes.to_channels(node.state, prev))
        result = yield ("eval",)
        evaluator.reply(node, *result)
        yield ("replied",)

    def yield_(self):
        yield ("yield",)

    def add_runnable(self, gen):
        self.runnables.append(gen)

    def create_main_loop(self):
        if self.main is None:
            self.main = self._main_loop()

    def _step(self, g, value=None):
        try:
            return g.send(value)
        except StopIteration:
            return ("dead",)

    def _main_loop(self):
        while True:
            jump = False
            if not self.runnables:
                if not self.requestors:
                    if self.yielders:
                        self.runnables.extend(self.yielders)
                        self.yielders = []
                        continue
                    break
                jump = True
            if not jump and len(self.requestors) == self.batch_size:
                jump = True
            if jump:
                yield "top"
                assert self.pde[0] == len(self.requestors)
                for idx, g in enumerate(self.requestors):
                    count, pols, vals = self.pde
                    policies = [np.asarray(p).reshape(-1)[idx * ps:(idx + 1) * ps] for p, ps in zip(pols, self.policy_sizes)]
                    rewards = np.asarray(vals).reshape(-1)[idx * self.num_rewards:(idx + 1) * self.num_rewards]
                    r = self._step(g, (policies, rewards))
                    assert r[0] == "replied"
                    self.runnables.append(g)
                self.requestors = []
                self.runnables.extend(self.yielders)
                self.yielders = []
            g = self.runnables.popleft()
            r = self._step(g)
            if r[0] == "eval":
                self.requestors.append(g)
            elif r[0] == "yield":
                self.yielders.append(g)

    def poll(self, pred_count, policies, values):
        self.pde = (pred_count, policies, values)
        self.buf = []
        try:
            next(self.main)
        except StopIteration:
            self.main = None
        if not self.buf:
            return None
        return np.concatenate(self.buf)


def parse_conf(conf):
    """attrs record or dict -> plain dict (missing keys keep confs.py defaults)."""
    import attr
    if not isinstance(conf, dict):
        conf = attr.asdict(conf)
    return dict(conf)


class UniqueStates(object):
    def __init__(self, mask, max_num_dupes=1000):
        self.mask = mask
        self.max_num_dupes = max_num_dupes
        self.lookup = {}

    def add(self, state):
        k = state & self.mask
        if k in self.lookup:
            if self.lookup[k] < self.max_num_dupes:
                self.lookup[k] += 1
            return
        self.lookup[k] = 1

    def is_unique(self, state, depth):
        k = state & self.mask
        if k in self.lookup:
            if self.lookup[k] >= max(2, self.max_num_dupes - 5 * depth):
                return False
        return True


class SelfPlay(object):
    """selfplay.cpp:29-343"""

    def __init__(self, manager, conf, pe, identifier, seed):
        self.manager = manager
        self.conf = conf
        self.pe = pe
        self.identifier = identifier
        self.match_count = 0
        self.rng = S.Rng(seed)
        self.game_samples = []

    def resign(self, node):
        score = node.current[node.lead_role_index]
        rc = self.manager.sm.role_count
        if self.can_resign0 and score < F32(self.conf["resign0_score_probability"]):
            self.has_resigned = True
            self.r0 = [node.current[i] for i in range(rc)]
        elif self.can_resign1 and score < F32(self.conf["resign1_score_probability"]):
            self.has_resigned = True
            self.r1 = [node.current[i] for i in range(rc)]

    def collect_samples(self, node):
        conf = self.conf
        self.pe.update_conf(conf["puct_config"])
        osc = float(F32(conf["oscillate_sampling_pct"]))
        evals = conf["evals_per_move"]
        man = self.manager.unique_states
        while True:
            if conf["abort_max_length"] > 0 and node.game_depth > conf["abort_max_length"]:
                break
            if node.is_terminal():
                break
            do_skip = False
            if not man.is_unique(node.state, node.game_depth):
                self.manager.stats["dupes"] += 1
                do_skip = True
            elif osc > 0 and self.rng.get() > osc:
                do_skip = True
            if not do_skip:
                man.add(node.state)
                self.pe.reset_root_node()
                choice = yield from self.pe.on_next_move(evals)
                self.pe.get_probabilities(node, F32(conf["temperature_for_policy"]), False)
                self.game_samples.append(self.manager.create_sample(node))
            else:
                skip_evals = max(16, self.rng.getWithMax(evals // 3 + 1))
                self.pe.update_conf(conf["run_to_end_puct_config"])
                choice = yield from self.pe.on_next_move(skip_evals)
                self.pe.update_conf(conf["puct_config"])
            node = yield from self.pe.fast_apply_move(choice)
            if node.is_terminal():
                break
            if not self.has_resigned:
                self.resign(node)
            if self.has_resigned and len(self.game_samples) > 1:
                self.manager.stats["resigns"] += 1
                break
        return node

    def run_to_end(self, node, final_scores):
        conf = self.conf
        self.pe.update_conf(conf["run_to_end_puct_config"])
        evals = conf["run_to_end_evals"]
        can = self.has_resigned and self.rng.get() > float(F32(conf["run_to_end_pct"]))

        def done(n):
            if conf["abort_max_length"] > 0 and n.game_depth > conf["abort_max_length"]:
                return True
            return n.is_finalised
        rc = self.manager.sm.role_count
        while not done(node):
            choice = yield from self.pe.on_next_move(evals)
            node = yield from self.pe.fast_apply_move(choice)
            if node.is_finalised:
                break
            if can and node.game_depth > conf["run_to_end_minimum_game_depth"]:
                if node.current[node.lead_role_index] < F32(conf["run_to_end_early_score"]):
                    self.manager.stats["early_run_to_ends"] += 1
                    for ri in range(rc):
                        final_scores.append(F32(0.0 if ri == node.lead_role_index else 1.0))
                    return node.game_depth
        if conf["abort_max_length"] > 0 and node.game_depth > conf["abort_max_length"]:
            return -1
        for ri in range(rc):
            final_scores.append(node.current[ri])
        return node.game_depth

    def play_once(self):
        conf = self.conf
        self.match_count += 1
        self.game_samples = []
        self.has_resigned = False
        r = self.rng.get()
        self.can_resign0 = r > float(F32(conf["resign0_pct"]))
        self.can_resign1 = r > float(F32(conf["resign1_pct"]))
        self.r0, self.r1 = [], []
        self.pe.reset(0)
        node = yield from self.pe.establish_root(None)
        start = node.game_depth
        node = yield from self.collect_samples(node)
        if not self.game_samples:
            self.manager.stats["no_samples"] += 1
            return
        final_scores = []
        game_depth = yield from self.run_to_end(node, final_scores)
        if game_depth == -1:
            self.manager.stats["aborts_game_length"] += 1
            return
        fp0 = fp1 = False
        for ri in range(self.manager.sm.role_count):
            fs = final_scores[ri]
            if self.has_resigned:
                for scores, prob_key, which in ((self.r0, "resign0_score_probability", 0),
                                                (self.r1, "resign1_score_probability", 1)):
                    if (fp0 if which == 0 else fp1):
                        continue
                    if scores and float(scores[ri]) < float(F32(conf[prob_key])) * 1.05 and float(fs) > 0.49:
                        if which == 0:
                            fp0 = True
                        else:
                            fp1 = True
        for s in self.game_samples:
            s["final_score"] = [float(x) for x in final_scores]
            s["game_length"] = game_depth
            s["match_identifier"] = "%s_%d" % (self.identifier, self.match_count)
            s["has_resigned"] = self.has_resigned
            s["resign_false_positive"] = fp0 or fp1
            s["starting_sample_depth"] = start
            self.manager.samples.append(s)

    def play_games_forever(self):
        while True:
            yield from self.play_once()


class Manager(object):
    """SelfPlayManager (selfplaymanager.cpp) for one pool, inline."""

    def __init__(self, sm, planes, batch_size, unique_states, identifier, seed, game_index_base,
                 policy_sizes, num_rewards, num_prev_states):
        self.sm = sm
        self.planes = planes
        self.batch_size = batch_size
        self.unique_states = unique_states
        self.identifier = identifier
        self.seed = seed
        self.game_index_base = game_index_base
        self.num_prev_states = num_prev_states
        self.scheduler = Scheduler(planes, batch_size, num_prev_states, policy_sizes, num_rewards)
        self.num_rewards = num_rewards
        self.samples = []
        self.stats = dict(dupes=0, resigns=0, no_samples=0, aborts_game_length=0, early_run_to_ends=0)
        self.evaluators = []
        self.self_plays = []

    def create_sample(self, node):
        rc = self.sm.role_count
        prev, cur = [], node.parent
        for _ in range(self.num_prev_states):
            if cur is None:
                break
            prev.append(cur.state)
            cur = cur.parent
        policies = []
        for ri in range(rc):
            pol = []
            for c in node.children:
                if ri == node.lead_role_index:
                    pol.append((c.move[ri], float(c.next_prob)))
                else:
                    pol.append((c.move[ri], 1.0))
                    break
            policies.append(pol)
        return dict(state=node.state, prev_states=prev, policies=policies, depth=node.game_depth,
                    resultant_puct_visits=node.visits,
                    resultant_puct_score=[float(node.current[i]) for i in range(rc)])

    def start(self, conf):
        conf = parse_conf(conf)
        conf["puct_config"] = parse_conf(conf["puct_config"])
        conf["run_to_end_puct_config"] = parse_conf(conf["run_to_end_puct_config"])
        self.conf = conf
        self.scheduler.create_main_loop()
        for ii in range(self.batch_size):
            gi = self.game_index_base + ii
            pe = Evaluator(self.sm, self.scheduler, self.planes, self.num_rewards)
            pe.update_conf(conf["puct_config"])
            pe.rng.seed(S.rng_mix(self.seed, gi, 0))
            self.evaluators.append(pe)
            sp = SelfPlay(self, conf, pe, "%s_%d" % (self.identifier, ii), S.rng_mix(self.seed, gi, 1))
            self.self_plays.append(sp)
            self.scheduler.add_runnable(sp.play_games_forever())

    def poll(self, pred_count, policies, values):
        return self.scheduler.poll(pred_count, policies, values)


class Player(object):
    """player.cpp:16-173 (match play: one evaluator, one scheduler)."""

    def __init__(self, sm, planes, conf, policy_sizes, num_rewards, num_prev_states, seed=0):
        self.sm = sm
        self.conf = parse_conf(conf)
        self.scheduler = Scheduler(planes, self.conf["batch_size"], num_prev_states, policy_sizes, num_rewards)
        self.evaluator = Evaluator(sm, self.scheduler, planes, num_rewards)
        self.evaluator.update_conf(self.conf)
        self.evaluator.rng.seed(S.rng_mix(seed, 0, 0))
        self.first_play = False
        self.choice = None

    def reset(self, game_depth=0):
        self.evaluator.reset(game_depth)
        self.first_play = True

    def move(self, state, evaluations):
        self.choice = None
        self.scheduler.create_main_loop()
        first = self.first_play
        self.first_play = False

        def run():
            if first:
                yield from self.evaluator.establish_root(state)
            self.choice = yield from self.evaluator.on_next_move(evaluations)
        self.scheduler.add_runnable(run())

    def apply_move(self, move):
        self.scheduler.create_main_loop()
        first = self.first_play
        self.first_play = False

        def run():
            if first:
                yield from self.evaluator.establish_root(None)
            yield from self.evaluator.apply_move(move)
        self.scheduler.add_runnable(run())

    def get_move(self, lead_role_index):
        if self.choice is None:
            return (-1, -1.0, -1)
        node = self.choice.to_node
        prob = float(node.current[lead_role_index]) if node is not None else -1.0
        return (self.choice.move[lead_role_index], prob, self.evaluator.number_of_nodes)

    def poll(self, pred_count, policies, values):
        if self.scheduler.main is None:
            return None
        return self.scheduler.poll(pred_count, policies, values)

    def root_children(self):
        root = self.evaluator.root
        lead = max(root.lead_role_index, 0)
        return [(c.move[lead], c.traversals, float(c.policy_prob)) for c in root.children]
