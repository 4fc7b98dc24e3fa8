package ai.foremast.metrics.boot1;

import org.springframework.boot.autoconfigure.condition.ConditionalOnClass;
import org.springframework.boot.autoconfigure.condition.ConditionalOnProperty;
import org.springframework.context.annotation.Configuration;
import org.springframework.core.annotation.Order;
import org.springframework.core.env.Environment;
import org.springframework.security.config.annotation.web.builders.HttpSecurity;
import org.springframework.security.config.annotation.web.configuration.WebSecurityConfigurerAdapter;

/**
 * With Spring Security on the classpath: the scrape, health / info and the
 * metric control paths are reachable without credentials, only them (the
 * reference 1.x starter's ActuatorSecurityConfig role).  {@code
 * k8s.metrics.disable-csrf=true} turns CSRF off for these paths (a POST to
 * /k8s-metrics/* from a script); {@code k8s.metrics.open-actuator=false}
 * leaves security to the application.
 */
@Configuration
@ConditionalOnClass(WebSecurityConfigurerAdapter.class)
@ConditionalOnProperty(prefix = "k8s.metrics", name = "open-actuator", havingValue = "true", matchIfMissing = true)
@Order(101)
public class Boot1ActuatorAccess extends WebSecurityConfigurerAdapter {

    static final String[] OPEN = {"/prometheus", "/actuator/prometheus", "/metrics", "/health", "/info",
        "/actuator/health", "/actuator/info", "/k8s-metrics/**"};

    private final boolean disableCsrf;

    public Boot1ActuatorAccess(Environment env) {
        super(true);                                  // no default configurers: only the paths below
        this.disableCsrf = "true".equalsIgnoreCase(env.getProperty("k8s.metrics.disable-csrf"));
    }

    @Override
    protected void configure(HttpSecurity http) throws Exception {
        http.requestMatchers().antMatchers(OPEN).and().authorizeRequests().anyRequest().permitAll();
        if (disableCsrf) {
            http.csrf().disable();
        }
    }
}
