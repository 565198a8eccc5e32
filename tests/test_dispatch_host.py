"""Host-side mirror of the reference's plugin surface (no GPU needed):
HOCON parsing, Dispatchers.lookup alias/FQCN resolution, Mailboxes.lookup,
typed selectors and Behaviors -> behaviour kinds."""
import pytest

from akka_amd.config import Config, ConfigurationException
from akka_amd.dispatch import (BoundedMailbox, Behaviors, DispatcherPrerequisites, Dispatchers, GpuDispatcher,
                               MailboxSelector, Mailboxes, NonBlockingBoundedMailbox, UnboundedMailbox,
                               SingleConsumerOnlyUnboundedMailbox)
from akka_amd.engine import Kind

CONF = """
# comment
my-app {
  gpu-dispatcher {
    type = "akka_amd.dispatch.GpuDispatcherConfigurator"
    throughput = 7
    mailbox-type = "akka.dispatch.BoundedMailbox"
    mailbox-capacity = 64
    mailbox-push-timeout-time = 0s
    actors = 1000
    state-words = 2
  }
  alias-1 = "my-app.gpu-dispatcher"
  alias-2 = "my-app.alias-1"
  loop-a = "my-app.loop-b"
  loop-b = "my-app.loop-a"
  fjp {
    type = Dispatcher
  }
  custom { type = "com.example.Nope" }
  deadline {
    type = "akka_amd.dispatch.GpuDispatcherConfigurator"
    throughput-deadline-time = 10ms
  }
}
bounded-mailbox {
  mailbox-type = "akka.dispatch.NonBlockingBoundedMailbox"
  mailbox-capacity = 16
}
blocking-mailbox {
  mailbox-type = "akka.dispatch.BoundedMailbox"
  mailbox-capacity = 16
  mailbox-push-timeout-time = 10s
}
my-app.dotted.key = 3
"""


def test_hocon_subset():
    c = Config.parse_string(CONF)
    assert c.get_int("my-app.gpu-dispatcher.throughput") == 7
    assert c.get_string("my-app.alias-1") == "my-app.gpu-dispatcher"
    assert c.get_int("my-app.dotted.key") == 3
    assert c.get_duration_s("my-app.deadline.throughput-deadline-time") == pytest.approx(0.01)
    merged = Config.parse_string("a { x = 1 }").with_fallback(Config.parse_string("a { x = 2, y = 3 }"))
    assert merged.get_int("a.x") == 1 and merged.get_int("a.y") == 3


def test_lookup_gpu_dispatcher_and_aliases():
    d = Dispatchers(Config.parse_string(CONF), DispatcherPrerequisites())
    disp = d.lookup("my-app.gpu-dispatcher")
    assert isinstance(disp, GpuDispatcher)
    assert disp.throughput == 7 and disp.mailbox_type == BoundedMailbox(64, 0.0)
    assert disp.id == "my-app.gpu-dispatcher"
    assert d.lookup("my-app.alias-2") is disp  # alias chain resolves to the same configurator
    assert not disp.is_throughput_deadline_time_defined()
    assert disp._engine is None  # engine (executor) created lazily, no GPU touched
    assert d.has_dispatcher("my-app.alias-1") and not d.has_dispatcher("nope")


def test_lookup_errors_match_reference():
    d = Dispatchers(Config.parse_string(CONF))
    with pytest.raises(ConfigurationException, match="not configured"):
        d.lookup("nope")
    with pytest.raises(ConfigurationException, match="loop"):
        d.lookup("my-app.loop-a")
    with pytest.raises(ConfigurationException, match="ForkJoinPool"):
        d.lookup("my-app.fjp")
    with pytest.raises(ConfigurationException, match="Cannot instantiate MessageDispatcherConfigurator"):
        d.lookup("my-app.custom")
    with pytest.raises(ConfigurationException, match="throughput-deadline-time"):
        d.lookup("my-app.deadline")


def test_mailboxes_lookup():
    m = Mailboxes(Config.parse_string(CONF))
    assert m.lookup("unbounded") == UnboundedMailbox()
    assert m.lookup("bounded") == BoundedMailbox(1000, 0.0)  # default-mailbox capacity (Mailboxes.scala:211)
    assert m.lookup(MailboxSelector.bounded(12)) == BoundedMailbox(12, 0.0)  # bounded-capacity:N
    assert m.lookup("bounded-mailbox") == NonBlockingBoundedMailbox(16)
    assert m.lookup("akka.actor.typed.default-mailbox") == SingleConsumerOnlyUnboundedMailbox()
    with pytest.raises(ConfigurationException, match="never block"):
        m.lookup("blocking-mailbox")
    with pytest.raises(ConfigurationException, match="not configured"):
        m.lookup("missing-mailbox")


def test_behaviors_map_to_kinds():
    assert Behaviors.counter().kind == Kind.COUNTER
    assert Behaviors.ring(3).params == ("ring", 3)
    assert Behaviors.stop_after(5).init == (0, 5) and Behaviors.stop_after(5).min_words == 2
    assert Behaviors.ping_pong(2_000_000).init == (1_000_000, 0)
    assert Behaviors.even_only().kind == Kind.EVEN


def test_bounded_capacity_validation():
    with pytest.raises(ValueError):
        BoundedMailbox(-1)
