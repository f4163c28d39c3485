"""PUCTPlayer: match play over PlayPoller (reference src/ggpzero/player/puctplayer.py:13-108).

The reference derives from ggplib's ``MatchPlayer`` and reads its match through ggplib objects
(``match.game_info``, ``match.get_current_state()``, ``match.our_role_index``,
``match.game_depth``).  ggplib is not part of this build, so :class:`Match` is the small stand-in
holding exactly those fields over the native state machines; the player's own methods keep the
reference's names, arguments and call order (player_reset at meta-gaming, apply_move + poll_loop,
move + poll_loop + get_move).  ``nn`` may be passed in directly instead of loading
``conf.generation`` through the manager (``manager.py:129-139``).
"""
from ..cppinterface import PlayPoller
from ..defs import confs
from ..sm import get_sm


class Match(object):
    """The fields of ggplib's match the player reads."""

    def __init__(self, game, our_role_index, match_id="match"):
        self.game = game
        self.sm = get_sm(game)
        self.our_role_index = our_role_index
        self.match_id = match_id
        self.state = self.sm.get_initial_state().copy()
        self.game_depth = 0

    def get_current_state(self):
        return self.state

    def apply(self, joint_move):
        self.sm.update_bases(self.state)
        self.state = self.sm.next_state(list(joint_move)).copy()
        self.game_depth += 1

    def is_terminal(self):
        self.sm.update_bases(self.state)
        return self.sm.is_terminal()


class PUCTPlayer(object):
    poller = None
    last_probability = -1
    last_node_count = -1

    def __init__(self, conf, nn=None, seed=0):
        assert isinstance(conf, (confs.PUCTPlayerConfig, confs.PUCTEvaluatorConfig))
        self.conf = conf
        if conf.playouts_per_iteration > 0:
            self.identifier = "%s_%s_%s" % (conf.name, conf.playouts_per_iteration, conf.generation)
        else:
            self.identifier = "%s_%s" % (conf.name, conf.generation)
        self.nn = nn
        self.seed = seed
        self.sm = None
        self.match = None

    def get_name(self):
        return self.identifier

    def cleanup(self):
        if self.poller is not None:
            self.poller.player_reset(0)

    def on_meta_gaming(self, finish_time=-1):
        """puctplayer.py:33-63.  As in ggplib's MatchPlayer, the match is set on the player
        (``player.match = ...``) before meta-gaming."""
        match = self.match
        assert match is not None, "set player.match before on_meta_gaming (MatchPlayer protocol)"
        if self.sm is None or "*" in self.conf.generation:
            self.sm = get_sm(match.game)
            if self.nn is None:
                from ..nn.manager import get_manager
                self.nn = get_manager().load_network(match.game, self.conf.generation)
            self.poller = PlayPoller(self.sm, self.nn, self.conf.evaluator_config, seed=self.seed)
            # role r is the noop-only role when the other one leads; noop is action 0 of the
            # native state machines (the reference searches the action names, :55-61)
            self.role0_noop_legal = self.role1_noop_legal = 0
        self.poller.player_reset(match.game_depth)

    def on_apply_move(self, joint_move):
        """puctplayer.py:65-67."""
        self.poller.player_apply_move(list(joint_move))
        self.poller.poll_loop()

    def on_next_move(self, finish_time=-1):
        """puctplayer.py:69-97: lead role from the noop-only role, iterations by whose turn it is."""
        current_state = self.match.get_current_state()
        self.sm.update_bases(current_state)
        l0 = self.sm.get_legal_state(0)
        if len(l0) == 1 and l0[0] == self.role0_noop_legal:
            lead_role_index = 1
        else:
            l1 = self.sm.get_legal_state(1)
            assert len(l1) == 1 and l1[0] == self.role1_noop_legal
            lead_role_index = 0
        if lead_role_index == self.match.our_role_index:
            max_iterations = self.conf.playouts_per_iteration
        else:
            max_iterations = self.conf.playouts_per_iteration_noop
        self.poller.player_move(current_state, max_iterations, finish_time)
        self.poller.poll_loop()
        move, prob, node_count = self.poller.player_get_move(self.match.our_role_index)
        self.last_probability = prob
        self.last_node_count = node_count
        return move

    def balance_moves(self, max_count):
        self.poller.player_balance_moves(max_count)
        self.poller.poll_loop()

    def tree_debug(self, max_count):
        return self.poller.player_tree_debug(max_count)

    def update_config(self, *args, **kwds):
        self.poller.player_update_config(*args, **kwds)

    def __repr__(self):
        return self.get_name()


def play_match(game, players, max_moves=500):
    """Plays players[0] (role 0) against players[1] (role 1) from the initial state; returns
    (goal values, moves).  Both players see every joint move (the GGP protocol's play message)."""
    matches = [Match(game, r) for r in range(2)]
    for p, m in zip(players, matches):
        p.match = m
        p.on_meta_gaming(-1)
    moves = []
    ref = matches[0]
    while not ref.is_terminal() and len(moves) < max_moves:
        joint = [players[r].on_next_move() for r in range(2)]
        moves.append(joint)
        for p, m in zip(players, matches):
            m.apply(joint)
            p.on_apply_move(joint)
    ref.sm.update_bases(ref.state)
    return [ref.sm.get_goal_value(r) for r in range(2)], moves
