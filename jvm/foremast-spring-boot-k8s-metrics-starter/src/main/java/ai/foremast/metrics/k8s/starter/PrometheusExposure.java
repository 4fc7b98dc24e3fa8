package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.SpringApplication;
import org.springframework.boot.env.EnvironmentPostProcessor;
import org.springframework.core.Ordered;
import org.springframework.core.env.ConfigurableEnvironment;
import org.springframework.core.env.MapPropertySource;

import java.util.Collections;
import java.util.LinkedHashSet;
import java.util.Set;

/**
 * Makes sure the actuator exposes what foremast needs over HTTP: the
 * {@code prometheus} scrape (Prometheus, the recording rules, the brain) and
 * the {@code k8s-metrics} gate toggle (kubectl plugins) -- added to
 * {@code management.endpoints.web.exposure.include} as the highest-priority
 * property source, on top of whatever the application lists there
 * ({@code health,info} when it lists nothing, Spring Boot's own default).
 * An application that excludes them explicitly
 * ({@code management.endpoints.web.exposure.exclude}) still wins: exclusion
 * is applied after inclusion by the actuator.  Registered in
 * META-INF/spring.factories (runs before any auto-configuration).
 */
public class PrometheusExposure implements EnvironmentPostProcessor, Ordered {

    static final String INCLUDE = "management.endpoints.web.exposure.include";

    @Override
    public void postProcessEnvironment(ConfigurableEnvironment env, SpringApplication application) {
        String cur = env.getProperty(INCLUDE, "");
        Set<String> ids = new LinkedHashSet<>(MeterGate.tokens(cur));
        if (ids.contains("*")) {
            return;                                   // everything is exposed already
        }
        if (ids.isEmpty()) {
            ids.add("health");
            ids.add("info");
        }
        ids.add("prometheus");
        ids.add("k8s-metrics");
        env.getPropertySources().addFirst(new MapPropertySource("foremastExposure",
                Collections.singletonMap(INCLUDE, String.join(",", ids))));
    }

    @Override
    public int getOrder() {
        return Ordered.LOWEST_PRECEDENCE;             // after the application's own config files are loaded
    }
}
