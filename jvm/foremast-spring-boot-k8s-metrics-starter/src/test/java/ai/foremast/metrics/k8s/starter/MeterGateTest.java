package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Meter;
import io.micrometer.core.instrument.Tags;
import io.micrometer.core.instrument.config.MeterFilterReply;
import org.junit.jupiter.api.Test;

import java.util.HashMap;
import java.util.Map;

import static org.junit.jupiter.api.Assertions.assertEquals;
import static org.junit.jupiter.api.Assertions.assertFalse;

/** The same cases as tests/test_emitter.py's CommonMetricsFilter checks. */
class MeterGateTest {

    private static Meter.Id id(String name, String... tags) {
        return new Meter.Id(name, Tags.of(tags), null, null, Meter.Type.COUNTER);
    }

    @Test
    void gateOrder() {
        K8sMetricsProperties p = new K8sMetricsProperties();
        p.setEnableCommonMetricsFilter(true);
        p.setEnableCommonMetricsFilterAction(true);
        p.setCommonMetricsWhitelist("jvm_memory_used_bytes");
        p.setCommonMetricsBlacklist("process_cpu_usage");
        p.setCommonMetricsPrefix("http.");
        p.setCommonMetricsTagRules("team:sre");
        Map<String, Boolean> enable = new HashMap<>();
        enable.put("tomcat", false);
        MeterGate g = new MeterGate(p, enable);
        assertEquals(MeterFilterReply.DENY, g.accept(id("tomcat.sessions.active")));
        assertEquals(MeterFilterReply.NEUTRAL, g.accept(id("jvm.memory.used")));
        assertEquals(MeterFilterReply.DENY, g.accept(id("process.cpu.usage")));
        assertEquals(MeterFilterReply.ACCEPT, g.accept(id("http.server.requests")));
        assertEquals(MeterFilterReply.ACCEPT, g.accept(id("queue.depth", "team", "sre")));
        assertEquals(MeterFilterReply.DENY, g.accept(id("queue.depth", "team", "web")));
        g.enableMetric("queue_depth");
        assertEquals(MeterFilterReply.NEUTRAL, g.accept(id("queue.depth")));
        g.disableMetric("queue_depth");
        assertEquals(MeterFilterReply.DENY, g.accept(id("queue.depth", "team", "sre")));
    }

    @Test
    void actionsOffByDefault() {
        MeterGate g = new MeterGate(new K8sMetricsProperties(), null);
        assertFalse(g.enableMetric("x"));
        assertEquals(MeterFilterReply.NEUTRAL, g.accept(id("anything")));
    }
}
